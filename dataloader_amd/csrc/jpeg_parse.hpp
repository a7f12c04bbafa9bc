// jpeg_parse.hpp — marker-segment parser for baseline/extended sequential JPEG.
//
// Restates what libjpeg-turbo (inside Pillow, the decoder the reference calls at
// cpu.py:251) does before the first scan: jdmarker.c (SOF/DHT/DQT/DRI/SOS/APPn),
// jdapimin.c default_decompress_parms (colour-space guess), jdinput.c
// initial_setup / per_scan_setup (component and MCU geometry).  Conditions on
// which libjpeg raises (and the reference therefore zero-fills, cpu.py:252)
// map to negative statuses; JPEG flavours libjpeg decodes but this backend
// does not map to positive statuses.
#pragma once

#include "common.hpp"

namespace dino {

// jpeg_natural_order + 16 safety entries (jutils.c): zigzag index -> natural index.
constexpr uint8_t kNaturalOrder[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

DHD int rd16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// Parse markers of one JPEG held in p[0..len).  Fills geometry, tables and the
// entropy-data offset.  Returns d->status.
// Pillow's DecompressionBombError threshold: 2 x Image.MAX_IMAGE_PIXELS (PIL/Image.py).
constexpr int64_t kPilBombPixels = 2ll * 89478485;

DHD uint32_t rd32le(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Size checks shared by both image kinds: Pillow refuses decompression bombs at
// Image.open (the reference then zero-fills).  The bomb limit also bounds every pixel
// index of the colour / resize kernels (3 x 2 x 89478485 bytes < 2^31), so any side the
// JPEG format allows (<= 65535) decodes; a caller-chosen side limit (max_dim < 65535)
// reports DINO_IMG_LIMIT for JPEGs, which the Python layer hands to Pillow.  Raw
// containers (already Pillow's output) are only bound by the bomb limit.
DHD int check_dims(ImgDesc* d, int max_dim) {
  if ((int64_t)d->width * d->height > kPilBombPixels) return (d->status = DINO_IMG_TOO_LARGE);
  if (d->kind != 2 && (d->width > max_dim || d->height > max_dim)) return (d->status = DINO_IMG_LIMIT);
  return d->status;
}

// allow_raw: the caller marked this image as a pre-decoded RGB container (raw mask of
// dino_decode / dino_probe).  The container's magic is never trusted in user data: an
// unmarked file that starts with it is parsed as what it is (not a JPEG -> corrupt, as
// Pillow would raise).
DHD int parse_jpeg(const uint8_t* p, int64_t len, int max_dim, ImgDesc* d, bool allow_raw = false) {
  d->status = DINO_IMG_CORRUPT;
  d->width = d->height = d->ncomp = 0;
  d->restart_interval = 0;
  d->scan_off = d->scan_len = 0;
  d->kind = 0;
  d->progressive = 0;
  d->first_sos = 0;
  d->n_scans = 0;
  d->qt_seen_mask = 0;
  d->aug_status = 0;
  d->rst_bad = 0;
  d->total_blocks = 0;
  for (int i = 0; i < 8; ++i) d->huff_off[i] = -1;
  for (int t = 0; t < 4; ++t)
    for (int k = 0; k < 64; ++k) d->qt[t][k] = 0;
  bool qt_seen[4] = {false, false, false, false};
  // pre-decoded RGB container (include/dino_ingest.h DINO_RAW_MAGIC)
  if (allow_raw) {
    if (len < 16 || rd32le(p) != DINO_RAW_MAGIC) return d->status;
    const uint32_t w = rd32le(p + 4), h = rd32le(p + 8);
    if (w < 1 || h < 1 || w > 65535 || h > 65535 || (int64_t)w * h * 3 > len - 16) return d->status;
    d->kind = 2;
    d->width = (int32_t)w;
    d->height = (int32_t)h;
    d->ncomp = 3;
    d->color = kRGB;
    d->scan_off = 16;
    d->scan_len = (int32_t)((int64_t)w * h * 3 > 0x7FFFFFFF ? 0x7FFFFFFF : (int64_t)w * h * 3);
    d->status = DINO_IMG_OK;
    return check_dims(d, max_dim);
  }
  // Pillow's _accept: the file must start with FF D8 FF
  if (len < 4 || p[0] != 0xFF || p[1] != 0xD8 || p[2] != 0xFF) return d->status;

  bool saw_sof = false, saw_jfif = false, saw_adobe = false;
  int adobe_transform = 0;
  int64_t pos = 2;
  for (;;) {
    // next_marker(): skip garbage up to 0xFF, then any fill 0xFFs
    while (pos < len && p[pos] != 0xFF) ++pos;
    while (pos < len && p[pos] == 0xFF) ++pos;
    if (pos >= len) return d->status;  // no SOS: Pillow raises
    int m = p[pos++];
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // standalone markers
    if (m == 0xD9) return d->status;                                    // EOI before SOS
    if (pos + 2 > len) return d->status;
    int seglen = rd16(p + pos);
    if (seglen < 2 || pos + seglen > len) return d->status;
    const uint8_t* s = p + pos + 2;
    int n = seglen - 2;
    switch (m) {
      case 0xC0:
      case 0xC1:
      case 0xC2: {  // SOF0 baseline / SOF1 extended sequential / SOF2 progressive, Huffman
        if (saw_sof || n < 6) return (d->status = DINO_IMG_CORRUPT);
        saw_sof = true;
        d->progressive = m == 0xC2;
        int prec = s[0];
        d->height = rd16(s + 1);
        d->width = rd16(s + 3);
        int nf = s[5];
        if (n < 6 + 3 * nf || nf <= 0) return (d->status = DINO_IMG_CORRUPT);
        // Pillow's SOF handler raises for precision != 8 and for layer counts other than
        // 1, 3, 4 (JpegImagePlugin.SOF): the reference zero-fills those
        if (prec != 8) return (d->status = DINO_IMG_CORRUPT);
        if (nf != 1 && nf != 3 && nf != 4) return (d->status = DINO_IMG_CORRUPT);
        if (nf == 4) return (d->status = DINO_IMG_UNSUPPORTED);  // CMYK / YCCK
        if (d->height == 0) return (d->status = DINO_IMG_UNSUPPORTED);  // DNL
        if (d->width == 0) return (d->status = DINO_IMG_CORRUPT);
        d->ncomp = nf;
        for (int c = 0; c < nf; ++c) {
          CompDesc& cd = d->comp[c];
          cd.id = s[6 + 3 * c];
          cd.h = s[7 + 3 * c] >> 4;
          cd.v = s[7 + 3 * c] & 15;
          cd.tq = s[8 + 3 * c];
          if (cd.h < 1 || cd.h > 4 || cd.v < 1 || cd.v > 4 || cd.tq > 3)
            return (d->status = DINO_IMG_BADDATA);
        }
        break;
      }
      case 0xC3: case 0xC5: case 0xC6: case 0xC7:
      case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        // lossless / hierarchical / arithmetic: left to the host (Pillow decides)
        if (n >= 1 && s[0] != 8) return (d->status = DINO_IMG_CORRUPT);  // Pillow: "cannot handle N-bit layers"
        return (d->status = DINO_IMG_UNSUPPORTED);
      case 0xCC:  // DAC: arithmetic coding
        return (d->status = DINO_IMG_UNSUPPORTED);
      case 0xC4: {  // DHT (may hold several tables)
        int q = 0;
        while (q < n) {
          if (q + 17 > n) return (d->status = DINO_IMG_CORRUPT);
          int tc = s[q] >> 4, th = s[q] & 15;
          int cnt = 0;
          for (int i = 1; i <= 16; ++i) cnt += s[q + i];
          if (cnt > 256 || q + 17 + cnt > n || tc > 1 || th > 3) return (d->status = DINO_IMG_CORRUPT);
          d->huff_off[tc * 4 + th] = (int32_t)(pos + 2 + q + 1);
          q += 17 + cnt;
        }
        break;
      }
      case 0xDB: {  // DQT
        int q = 0;
        while (q < n) {
          int pq = s[q] >> 4, tq = s[q] & 15;
          if (tq > 3 || pq > 1) return (d->status = DINO_IMG_CORRUPT);
          int need = pq ? 128 : 64;
          if (q + 1 + need > n) return (d->status = DINO_IMG_CORRUPT);
          for (int k = 0; k < 64; ++k) {
            int v = pq ? rd16(s + q + 1 + 2 * k) : s[q + 1 + k];
            d->qt[tq][kNaturalOrder[k]] = (uint16_t)v;
          }
          qt_seen[tq] = true;
          q += 1 + need;
        }
        break;
      }
      case 0xDD:  // DRI
        if (n < 2) return (d->status = DINO_IMG_CORRUPT);
        d->restart_interval = rd16(s);
        break;
      case 0xE0:  // APP0: JFIF?
        if (n >= 5 && s[0] == 'J' && s[1] == 'F' && s[2] == 'I' && s[3] == 'F' && s[4] == 0) saw_jfif = true;
        break;
      case 0xEE:  // APP14: Adobe transform flag
        if (n >= 12 && s[0] == 'A' && s[1] == 'd' && s[2] == 'o' && s[3] == 'b' && s[4] == 'e') {
          saw_adobe = true;
          adobe_transform = s[11];
        }
        break;
      case 0xDA: {  // SOS
        if (!saw_sof || n < 1) return (d->status = DINO_IMG_CORRUPT);
        int ns = s[0];
        if (n < 4 + 2 * ns || ns < 1 || ns > 4) return (d->status = DINO_IMG_CORRUPT);
        // One interleaved scan of every component in frame order decodes on the
        // baseline path; anything else (progressive, components spread over several
        // scans, another component order) on the coefficient-buffer path (k_prog),
        // whose marker walk re-reads this SOS.
        d->first_sos = (int32_t)(pos - 2);  // (a baseline image may still move to k_prog, k_destuff_write)
        bool one_scan = !d->progressive && ns == d->ncomp;
        for (int k = 0; k < ns && one_scan; ++k) {
          int cs = s[1 + 2 * k];
          int ci = -1;
          for (int c = 0; c < d->ncomp; ++c)
            if (d->comp[c].id == cs) ci = c;
          if (ci != k) one_scan = false;
        }
        if (!one_scan) {
          d->kind = 1;
          d->scan_off = (int32_t)(pos + seglen);
          d->scan_len = (int32_t)(len - d->scan_off);
          goto have_scan;
        }
        for (int k = 0; k < ns; ++k) {
          int t = s[2 + 2 * k];
          d->comp[k].td = t >> 4;
          d->comp[k].ta = t & 15;
          if (d->comp[k].td > 3 || d->comp[k].ta > 3) return (d->status = DINO_IMG_CORRUPT);
        }
        // Ss/Se/Ah/Al of a sequential scan are ignored (libjpeg: JWRN_NOT_SEQUENTIAL warning)
        d->scan_off = (int32_t)(pos + seglen);
        d->scan_len = (int32_t)(len - d->scan_off);
        goto have_scan;
      }
      default:
        break;  // APPn, COM, other: skipped
    }
    pos += seglen;
  }

have_scan:
  d->status = DINO_IMG_OK;
  if (check_dims(d, max_dim) != DINO_IMG_OK) return d->status;
  d->status = DINO_IMG_CORRUPT;
  for (int t = 0; t < 4; ++t) d->qt_seen_mask |= qt_seen[t] ? 1 << t : 0;
  if (d->kind == 0) {  // (kind 1: tables and quant latching are checked per scan by prog_walk)
    for (int c = 0; c < d->ncomp; ++c) {
      const CompDesc& cd = d->comp[c];
      if (!qt_seen[cd.tq]) return (d->status = DINO_IMG_CORRUPT);  // libjpeg JERR_NO_QUANT_TABLE
      if (d->huff_off[cd.td] < 0 || d->huff_off[4 + cd.ta] < 0)
        return (d->status = DINO_IMG_CORRUPT);                      // JERR_NO_HUFF_TABLE
    }
  }
  // colour space (jdapimin.c default_decompress_parms)
  if (d->ncomp == 1) {
    d->color = kGray;
  } else if (saw_jfif) {
    d->color = kYCbCr;
  } else if (saw_adobe) {
    d->color = adobe_transform == 0 ? kRGB : kYCbCr;
  } else if (d->comp[0].id == 82 && d->comp[1].id == 71 && d->comp[2].id == 66) {
    d->color = kRGB;
  } else {
    d->color = kYCbCr;
  }
  // geometry (jdinput.c initial_setup / per_scan_setup)
  int mh = 1, mv = 1;
  for (int c = 0; c < d->ncomp; ++c) {
    mh = d->comp[c].h > mh ? d->comp[c].h : mh;
    mv = d->comp[c].v > mv ? d->comp[c].v : mv;
  }
  d->max_h = mh;
  d->max_v = mv;
  for (int c = 0; c < d->ncomp; ++c) {
    CompDesc& cd = d->comp[c];
    // jdsample.c: only integral upsampling ratios are implemented
    if (mh % cd.h != 0 || mv % cd.v != 0) return (d->status = DINO_IMG_BADDATA);
    cd.dw = (int32_t)(((int64_t)d->width * cd.h + mh - 1) / mh);
    cd.dh = (int32_t)(((int64_t)d->height * cd.v + mv - 1) / mv);
  }
  if (d->ncomp == 1) {
    CompDesc& cd = d->comp[0];
    d->mcus_x = ceil_div(cd.dw, 8);
    d->mcus_y = ceil_div(cd.dh, 8);
    d->blocks_per_mcu = 1;
    cd.bw = d->mcus_x;
    cd.bh = d->mcus_y;
    d->mcu_comp[0] = 0;
    d->mcu_bx[0] = 0;
    d->mcu_by[0] = 0;
  } else {
    d->mcus_x = ceil_div(d->width, 8 * mh);
    d->mcus_y = ceil_div(d->height, 8 * mv);
    int b = 0;
    for (int c = 0; c < d->ncomp; ++c) {
      CompDesc& cd = d->comp[c];
      if (b + cd.h * cd.v > kMaxBlocksPerMcu) return (d->status = DINO_IMG_BADDATA);
      for (int y = 0; y < cd.v; ++y)
        for (int x = 0; x < cd.h; ++x) {
          d->mcu_comp[b] = (uint8_t)c;
          d->mcu_bx[b] = (uint8_t)x;
          d->mcu_by[b] = (uint8_t)y;
          ++b;
        }
      cd.bw = d->mcus_x * cd.h;
      cd.bh = d->mcus_y * cd.v;
    }
    d->blocks_per_mcu = b;
  }
  int64_t mcus = (int64_t)d->mcus_x * d->mcus_y;
  d->total_blocks = (int32_t)(mcus * d->blocks_per_mcu);
  d->n_rst_max = d->restart_interval > 0 ? (int32_t)((mcus + d->restart_interval - 1) / d->restart_interval) : 0;
  int64_t co = 0, po = 0;
  for (int c = 0; c < d->ncomp; ++c) {
    CompDesc& cd = d->comp[c];
    cd.coef_off = co;
    cd.plane_off = po;
    co += (int64_t)cd.bw * cd.bh * 128;
    po += (int64_t)cd.bw * cd.bh * 64;
  }
  d->coef_bytes = co;
  d->status = DINO_IMG_OK;
  return d->status;
}

// Per-image workspace sizes (bytes), used by k_plan.
DHD int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

}  // namespace dino
