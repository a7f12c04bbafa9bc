"""A small JPEG encoder for test data (TEST INFRASTRUCTURE ONLY).

Pillow can only write libjpeg's default scan scripts (one interleaved sequential scan,
or jpeg_simple_progression).  The decoders under test (the GPU coefficient-buffer path
k_prog and its host model) must also handle what other encoders write: sequential
files whose components arrive in separate (or partially interleaved) scans, scan
component orders that differ from the frame's, progressive scripts with other band
splits and deeper successive approximation, restart intervals that change between
scans, Huffman tables redefined or reused between scans, scripts that leave
coefficients unrefined (libjpeg then block-smooths).  This module writes such files;
the tests compare every decoder against Pillow/libjpeg-turbo decoding the same bytes,
so the encoder only has to be *valid*, not identical to any particular encoder.

Follows ITU-T T.81 (F.1 sequential, G.1 progressive) and libjpeg's jcphuff.c for the
progressive refinement coding (correction-bit buffering, EOB runs) and jchuff.c
jpeg_gen_optimal_table for the per-scan Huffman tables.
"""

from __future__ import annotations

import numpy as np

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])  # zigzag index -> natural index

STD_LUMA_Q = np.array([
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
    14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99])  # natural order
STD_CHROMA_Q = np.array([
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
    47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32)


def quant_table(base: np.ndarray, quality: int) -> np.ndarray:
    """libjpeg jpeg_quality_scaling + jpeg_add_quant_table (force_baseline)."""
    q = max(1, min(100, quality))
    scale = 5000 // q if q < 50 else 200 - 2 * q
    t = (base * scale + 50) // 100
    return np.clip(t, 1, 255).astype(np.int64)


def _dct_matrix() -> np.ndarray:
    c = np.zeros((8, 8))
    for u in range(8):
        for x in range(8):
            c[u, x] = (np.sqrt(0.5) if u == 0 else 1.0) * np.cos((2 * x + 1) * u * np.pi / 16) / 2
    return c


_C = _dct_matrix()


def _component_coefs(plane: np.ndarray, bw: int, bh: int, q: np.ndarray) -> np.ndarray:
    """Quantized DCT coefficients [bh, bw, 64] (natural order) of a sample plane padded to bw x bh blocks."""
    h, w = plane.shape
    pad = np.pad(plane.astype(np.float64), ((0, bh * 8 - h), (0, bw * 8 - w)), mode="edge") - 128.0
    blocks = pad.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3)
    f = np.einsum("ux,abxy,vy->abuv", _C, blocks, _C)
    return np.round(f.reshape(bh, bw, 64) / q).astype(np.int64)


# ---- Huffman tables ---------------------------------------------------------------
def optimal_table(freq: np.ndarray) -> tuple[list[int], list[int]]:
    """jchuff.c jpeg_gen_optimal_table: (BITS[16], HUFFVAL) from symbol frequencies."""
    f = np.zeros(257, np.int64)
    f[:256] = freq
    f[256] = 1  # reserve one code point (no all-ones code)
    codesize = np.zeros(257, np.int64)
    others = -np.ones(257, np.int64)
    while True:
        c1, v = -1, 1 << 62
        for i in range(257):
            if f[i] and f[i] <= v:
                v, c1 = f[i], i
        c2, v = -1, 1 << 62
        for i in range(257):
            if f[i] and f[i] <= v and i != c1:
                v, c2 = f[i], i
        if c2 < 0:
            break
        f[c1] += f[c2]
        f[c2] = 0
        codesize[c1] += 1
        while others[c1] >= 0:
            c1 = others[c1]
            codesize[c1] += 1
        others[c1] = c2
        codesize[c2] += 1
        while others[c2] >= 0:
            c2 = others[c2]
            codesize[c2] += 1
    bits = np.zeros(40, np.int64)
    for i in range(257):
        if codesize[i]:
            bits[codesize[i]] += 1
    for i in range(39, 16, -1):
        while bits[i] > 0:
            j = i - 2
            while bits[j] == 0:
                j -= 1
            bits[i] -= 2
            bits[i - 1] += 1
            bits[j + 1] += 2
            bits[j] -= 1
    i = 16
    while bits[i] == 0:
        i -= 1
    bits[i] -= 1
    vals = [s for ln in range(1, 33) for s in range(256) if codesize[s] == ln]
    return [int(b) for b in bits[1:17]], vals


def canonical_codes(bits: list[int], vals: list[int]) -> dict[int, tuple[int, int]]:
    codes, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            codes[vals[k]] = (code, ln)
            code += 1
            k += 1
        code <<= 1
    return codes


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def bits(self, v: int, n: int):
        for i in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc = self.n = 0

    def flush(self):  # pad with 1 bits (T.81 F.1.2.3)
        if self.n:
            self.bits((1 << (8 - self.n)) - 1, 8 - self.n)


def _nbits(v: int) -> int:
    return int(abs(v)).bit_length()


def _extra(v: int, n: int) -> int:
    return v if v >= 0 else v + (1 << n) - 1


# ---- scan coding ---------------------------------------------------------------------
class _ScanCoder:
    """Codes one scan twice: a counting pass (symbol statistics -> optimal tables) and an
    emitting pass with those tables.  Symbols go to table slots ('dc', k) / ('ac', k)."""

    def __init__(self, emit: bool, tables=None):
        self.emit = emit
        self.tables = tables or {}
        self.freq: dict = {}
        self.w = BitWriter()

    def sym(self, slot, s: int):
        if self.emit:
            code, ln = self.tables[slot][s]
            self.w.bits(code, ln)
        else:
            self.freq.setdefault(slot, np.zeros(256, np.int64))[s] += 1

    def raw(self, v: int, n: int):
        if self.emit and n:
            self.w.bits(v, n)


def _scan_blocks(frame, scan):
    """(mcu index, [(scan component k, component c, by, bx)]) in coding order (jdinput per_scan_setup)."""
    comps = scan["comps"]
    if len(comps) == 1:
        c = comps[0]
        dw, dh = frame["dims"][c]
        bw, bh = -(-dw // 8), -(-dh // 8)
        for by in range(bh):
            for bx in range(bw):
                yield by * bw + bx, [(0, c, by, bx)]
    else:
        mx, my = frame["mcus"]
        for m in range(mx * my):
            mby, mbx = divmod(m, mx)
            blist = []
            for k, c in enumerate(comps):
                h, v = frame["samp"][c]
                for y in range(v):
                    for x in range(h):
                        blist.append((k, c, mby * v + y, mbx * h + x))
            yield m, blist


def _code_scan(frame, coefs, scan, coder: _ScanCoder, ri: int):
    ss, se, ah, al = scan["ss"], scan["se"], scan["ah"], scan["al"]
    prog = frame["progressive"]
    nk = len(scan["comps"])
    last_dc = [0] * nk
    eobrun, be = 0, []
    segments = []  # restart segments (bytes) when emitting

    def emit_eobrun():
        nonlocal eobrun, be
        if eobrun > 0:
            nb = eobrun.bit_length() - 1
            coder.sym(("ac", 0), nb << 4)
            coder.raw(eobrun, nb)
            eobrun = 0
            for bit in be:
                coder.raw(bit, 1)
            be = []

    def restart():
        nonlocal last_dc, eobrun, be
        emit_eobrun()
        if coder.emit:
            coder.w.flush()
            segments.append(bytes(coder.w.out))
            coder.w = BitWriter()
        last_dc = [0] * nk

    mcu_no = 0
    for m, blist in _scan_blocks(frame, scan):
        if ri and mcu_no and mcu_no % ri == 0:
            restart()
        mcu_no += 1
        for k, c, by, bx in blist:
            blk = coefs[c][by, bx]
            if not prog:  # sequential: DC + AC
                dc = int(blk[0])
                d = dc - last_dc[k]
                last_dc[k] = dc
                n = _nbits(d)
                coder.sym(("dc", k), n)
                coder.raw(_extra(d, n), n)
                r = 0
                for z in range(1, 64):
                    v = int(blk[ZIGZAG[z]])
                    if v == 0:
                        r += 1
                        continue
                    while r > 15:
                        coder.sym(("ac", k), 0xF0)
                        r -= 16
                    n = _nbits(v)
                    coder.sym(("ac", k), (r << 4) | n)
                    coder.raw(_extra(v, n), n)
                    r = 0
                if r:
                    coder.sym(("ac", k), 0x00)
            elif ss == 0 and ah == 0:  # DC first
                dc = int(blk[0]) >> al
                d = dc - last_dc[k]
                last_dc[k] = dc
                n = _nbits(d)
                coder.sym(("dc", k), n)
                coder.raw(_extra(d, n), n)
            elif ss == 0:  # DC refine
                coder.raw((int(blk[0]) >> al) & 1, 1)
            elif ah == 0:  # AC first (jcphuff encode_mcu_AC_first)
                r = 0
                for z in range(ss, se + 1):
                    v = int(blk[ZIGZAG[z]])
                    t = (-v >> al) if v < 0 else (v >> al)
                    if t == 0:
                        r += 1
                        continue
                    emit_eobrun()
                    while r > 15:
                        coder.sym(("ac", 0), 0xF0)
                        r -= 16
                    n = t.bit_length()
                    coder.sym(("ac", 0), (r << 4) | n)
                    coder.raw(t if v >= 0 else (~t) & ((1 << n) - 1), n)
                    r = 0
                if r > 0:
                    eobrun += 1
                    if eobrun == 0x7FFF:
                        emit_eobrun()
            else:  # AC refine (jcphuff encode_mcu_AC_refine)
                absv = [0] * 64
                eob = 0
                for z in range(ss, se + 1):
                    v = int(blk[ZIGZAG[z]])
                    t = abs(v) >> al
                    absv[z] = t
                    if t == 1:
                        eob = z
                r, br = 0, []
                for z in range(ss, se + 1):
                    t = absv[z]
                    if t == 0:
                        r += 1
                        continue
                    while r > 15 and z <= eob:
                        emit_eobrun()
                        coder.sym(("ac", 0), 0xF0)
                        r -= 16
                        for bit in br:
                            coder.raw(bit, 1)
                        br = []
                    if t > 1:
                        br.append(t & 1)
                        continue
                    emit_eobrun()
                    coder.sym(("ac", 0), (r << 4) | 1)
                    coder.raw(0 if int(blk[ZIGZAG[z]]) < 0 else 1, 1)
                    for bit in br:
                        coder.raw(bit, 1)
                    br = []
                    r = 0
                if r > 0 or br:
                    eobrun += 1
                    be += br
                    if eobrun == 0x7FFF or len(be) > 1000 - 64 + 1:
                        emit_eobrun()
    emit_eobrun()
    if coder.emit:
        coder.w.flush()
        segments.append(bytes(coder.w.out))
    return segments


# ---- file assembly --------------------------------------------------------------------
def _seg(marker: int, payload: bytes) -> bytes:
    return bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload


def _rgb_to_ycc(rgb: np.ndarray) -> np.ndarray:
    r, g, b = [rgb[..., i].astype(np.float64) for i in range(3)]
    y = 0.299 * r + 0.587 * g + 0.114 * b
    cb = -0.168736 * r - 0.331264 * g + 0.5 * b + 128
    cr = 0.5 * r - 0.418688 * g - 0.081312 * b + 128
    return np.clip(np.round(np.stack([y, cb, cr], -1)), 0, 255)


def encode(img: np.ndarray, scans: list[dict], quality: int = 85, samp=((2, 2), (1, 1), (1, 1)),
           progressive: bool = False, restart=None, comp_ids=(1, 2, 3), jfif: bool = True,
           before_scan: dict | None = None, coef_hook=None) -> bytes:
    """Encode ``img`` (H x W x 3 RGB or H x W gray) with an explicit scan script.

    scans: [{"comps": (frame component indices in scan order), "ss", "se", "ah", "al"}];
    for sequential files ss/se/ah/al are written as 0/63/0/0.  ``restart``: None, an int
    (one DRI before the first scan) or a list with one restart interval per scan (a DRI
    segment before each scan whose interval changes).  One DHT per scan (optimal tables).
    ``before_scan``: {scan index: raw marker segments inserted before that scan's tables}.
    ``coef_hook(coefs, qts) -> (coefs, qts)``: replaces the quantized coefficients
    ([bh, bw, 64] natural order per component) and quantization tables (<= 255) before
    coding, for tests that need chosen coefficient values.
    """
    gray = img.ndim == 2
    planes_full = [img.astype(np.float64)] if gray else list(np.moveaxis(_rgb_to_ycc(img), -1, 0))
    nc = len(planes_full)
    samp = samp[:nc] if not gray else ((1, 1),)
    H, W = planes_full[0].shape
    mh, mv = max(s[0] for s in samp), max(s[1] for s in samp)
    mx, my = -(-W // (8 * mh)), -(-H // (8 * mv))
    dims, coefs, qts = [], [], []
    for c in range(nc):
        h, v = samp[c]
        dw, dh = -(-W * h // mh), -(-H * v // mv)
        p = planes_full[c]
        fh, fv = mh // h, mv // v
        if fh > 1 or fv > 1:
            pp = np.pad(p, ((0, (-H) % fv), (0, (-W) % fh)), mode="edge")
            p = pp.reshape(pp.shape[0] // fv, fv, pp.shape[1] // fh, fh).mean(axis=(1, 3))
        p = np.clip(np.round(p), 0, 255)[:dh, :dw]
        q = quant_table(STD_LUMA_Q if c == 0 else STD_CHROMA_Q, quality)
        bw, bh = (mx * h, my * v) if nc > 1 else (-(-dw // 8), -(-dh // 8))
        coefs.append(_component_coefs(p, bw, bh, q))
        dims.append((dw, dh))
        qts.append(q)
    if coef_hook is not None:
        coefs, qts = coef_hook(coefs, qts)
    frame = {"dims": dims, "samp": list(samp), "mcus": (mx, my), "progressive": progressive}
    out = bytearray(b"\xff\xd8")
    if jfif:
        out += _seg(0xE0, b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00")
    nq = 1 if nc == 1 else 2
    for t in range(nq):
        out += _seg(0xDB, bytes([t]) + bytes(int(qts[0 if t == 0 else 1][ZIGZAG[z]]) for z in range(64)))
    sof = 0xC2 if progressive else 0xC0
    payload = bytes([8]) + H.to_bytes(2, "big") + W.to_bytes(2, "big") + bytes([nc])
    for c in range(nc):
        payload += bytes([comp_ids[c], (samp[c][0] << 4) | samp[c][1], 0 if c == 0 else 1])
    out += _seg(sof, payload)
    ris = restart if isinstance(restart, list) else [restart or 0] * len(scans)
    cur_ri = None
    for si, scan in enumerate(scans):
        ri = ris[si]
        if before_scan and si in before_scan:
            out += before_scan[si]
        if ri != cur_ri and (ri or cur_ri is not None):
            out += _seg(0xDD, int(ri).to_bytes(2, "big"))
            cur_ri = ri
        counter = _ScanCoder(False)
        _code_scan(frame, coefs, scan, counter, ri)
        tables, dht = {}, bytearray()
        slot_ids = {}
        for slot in sorted(counter.freq, key=lambda s: (s[0], s[1])):
            kind, k = slot
            tid = k % 4
            slot_ids[slot] = tid
            bits, vals = optimal_table(counter.freq[slot])
            dht += bytes([(0 if kind == "dc" else 16) | tid]) + bytes(bits) + bytes(vals)
            tables[slot] = canonical_codes(bits, vals)
        if dht:
            out += _seg(0xC4, bytes(dht))
        emitter = _ScanCoder(True, tables)
        segs = _code_scan(frame, coefs, scan, emitter, ri)
        comps = scan["comps"]
        sos = bytes([len(comps)])
        for k, c in enumerate(comps):
            td = slot_ids.get(("dc", k), 0)
            ta = slot_ids.get(("ac", 0 if progressive else k), 0)
            sos += bytes([comp_ids[c], (td << 4) | ta])
        if progressive:
            sos += bytes([scan["ss"], scan["se"], (scan["ah"] << 4) | scan["al"]])
        else:
            sos += bytes([0, 63, 0])
        out += _seg(0xDA, sos)
        for i, s in enumerate(segs):
            out += s
            if i + 1 < len(segs):
                out += bytes([0xFF, 0xD0 + (i % 8)])
    out += b"\xff\xd9"
    return bytes(out)


def scan(comps, ss=0, se=63, ah=0, al=0) -> dict:
    return {"comps": tuple(comps), "ss": ss, "se": se, "ah": ah, "al": al}


# Scripts used by the tests.
def sequential_per_component(nc: int = 3) -> list[dict]:
    return [scan((c,)) for c in range(nc)]


def simple_progression(nc: int = 3) -> list[dict]:
    """libjpeg jpeg_simple_progression (YCbCr)."""
    if nc == 1:
        return [scan((0,), 0, 0, 0, 1), scan((0,), 1, 5, 0, 2), scan((0,), 6, 63, 0, 2), scan((0,), 1, 63, 2, 1),
                scan((0,), 0, 0, 1, 0), scan((0,), 1, 63, 1, 0)]
    return [scan((0, 1, 2), 0, 0, 0, 1), scan((0,), 1, 5, 0, 2), scan((2,), 1, 63, 0, 1), scan((1,), 1, 63, 0, 1),
            scan((0,), 6, 63, 0, 2), scan((0,), 1, 63, 2, 1), scan((0, 1, 2), 0, 0, 1, 0), scan((2,), 1, 63, 1, 0),
            scan((1,), 1, 63, 1, 0), scan((0,), 1, 63, 1, 0)]


def deep_progression() -> list[dict]:
    """Non-interleaved DC scans, four successive-approximation levels, narrow bands."""
    return [scan((0,), 0, 0, 0, 2), scan((1,), 0, 0, 0, 0), scan((2,), 0, 0, 0, 1),
            scan((0,), 1, 2, 0, 3), scan((0,), 3, 9, 0, 3), scan((0,), 10, 63, 0, 3), scan((1,), 1, 63, 0, 0),
            scan((2,), 1, 63, 0, 2), scan((0,), 1, 63, 3, 2), scan((0,), 0, 0, 2, 1), scan((0,), 1, 63, 2, 1),
            scan((2,), 1, 63, 2, 1), scan((0,), 0, 0, 1, 0), scan((2,), 0, 0, 1, 0), scan((0,), 1, 63, 1, 0),
            scan((2,), 1, 63, 1, 0)]


def dqt_segment(table_id: int, quality: int, chroma: bool = False) -> bytes:
    q = quant_table(STD_CHROMA_Q if chroma else STD_LUMA_Q, quality)
    return _seg(0xDB, bytes([table_id]) + bytes(int(q[ZIGZAG[z]]) for z in range(64)))


def unrefined_progression() -> list[dict]:
    """A script that never refines the low AC coefficients to full precision: libjpeg
    block-smooths such images (jdcoefct.c smoothing_ok)."""
    return [scan((0, 1, 2), 0, 0, 0, 0), scan((0,), 1, 63, 0, 1), scan((1,), 1, 63, 0, 0), scan((2,), 1, 63, 0, 0)]
