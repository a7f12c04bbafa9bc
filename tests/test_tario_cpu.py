"""Host-side shard ingest (native tar index, gather, /dev/shm cache, batch feeder) on CPU.

The oracle for the tar walk is Python's ``tarfile`` plus WebDataset's key rule
(``base_plus_ext``), applied to shards built like the reference's fixtures
(``tests/fixtures/__init__.py:80-139``: ``sample_%06d.jpg`` + ``.json`` sidecars).
"""

from __future__ import annotations

import hashlib
import io
import json
import re
import struct
import tarfile

import numpy as np
import pytest
import torch

from dataloader_amd import tario


def _add(tf: tarfile.TarFile, name: str, data: bytes) -> None:
    ti = tarfile.TarInfo(name)
    ti.size = len(data)
    tf.addfile(ti, io.BytesIO(data))


def make_shard(n: int, with_meta: bool = True, fmt=tarfile.GNU_FORMAT, seed: int = 0, prefix: str = "") -> bytes:
    """Reference-fixture-shaped shard: JPEG-like payloads of varied length + JSON sidecars."""
    rng = np.random.default_rng(seed)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w", format=fmt) as tf:
        for i in range(n):
            key = f"{prefix}sample_{i:06d}"
            body = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
            _add(tf, f"{key}.jpg", b"\xff\xd8" + body + b"\xff\xd9")
            if with_meta:
                _add(tf, f"{key}.json", json.dumps({"quality_score": float(i % 5) / 4,
                                                    "caption": f"A test image number {i}"}).encode())
    return buf.getvalue()


_KEY_RE = re.compile(r"^((?:.*/|)[^.]+)[.]([^/]*)$")  # webdataset base_plus_ext


def oracle_samples(tar: bytes) -> list[tuple[str, bytes, bytes | None]]:
    """tarfile walk + WebDataset grouping: (key, jpeg bytes, json bytes or None)."""
    out: list[tuple[str, dict]] = []
    with tarfile.open(fileobj=io.BytesIO(tar), mode="r") as tf:
        for m in tf:
            if not m.isfile():
                continue
            mt = _KEY_RE.match(m.name)
            if not mt:
                continue
            key, ext = mt.group(1), mt.group(2).lower()
            if not out or out[-1][0] != key:
                out.append((key, {}))
            out[-1][1][ext] = tf.extractfile(m).read()
    res = []
    for key, d in out:
        img = d.get("jpg", d.get("jpeg"))
        if img is not None:
            res.append((key, img, d.get("json")))
    return res


def _index_via_file(tar: bytes) -> tario.TarIndex:
    """dino_tar_index_fd over the bytes written after a 16-byte shard-cache header."""
    import tempfile
    with tempfile.TemporaryFile() as f:
        f.write(b"H" * 16 + tar)
        f.flush()
        return tario.index_tar_fd(f.fileno(), 16, len(tar))


@pytest.fixture(params=["memory", "fd"])
def index_any(request):
    """Both forms of the tar walk: over mapped bytes, and over a file reading headers only."""
    return tario.index_tar if request.param == "memory" else _index_via_file


@pytest.mark.parametrize("fmt", [tarfile.GNU_FORMAT, tarfile.PAX_FORMAT, tarfile.USTAR_FORMAT])
@pytest.mark.parametrize("prefix", ["", "d" * 140 + "/"])
def test_tar_index_matches_tarfile(fmt, prefix, index_any):
    tar = make_shard(37, fmt=fmt, seed=3, prefix=prefix)
    idx = index_any(tar)
    ref = oracle_samples(tar)
    assert idx.status == 0 and len(idx) == len(ref) == 37
    assert idx.n_members == 74
    for row, key, (rk, rimg, rjson) in zip(idx.samples, idx.keys, ref):
        assert key == rk
        assert tar[row["img_off"]:row["img_off"] + row["img_len"]] == rimg
        assert tar[row["meta_off"]:row["meta_off"] + row["meta_len"]] == rjson


def test_tar_index_grouping_edge_cases(index_any):
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tf:
        _add(tf, "a.json", b"{}")                # sample without an image: skipped
        _add(tf, "b.JPEG", b"B")                 # extension lower-cased
        _add(tf, "noext", b"?")                  # no dot: not a sample member
        _add(tf, "dir/c.seg.jpg", b"C")          # key up to the first dot of the basename
        _add(tf, "dir/c.jpg", b"C2")             # same key, other extension
        _add(tf, ".hidden.jpg", b"H")            # basename starting with '.': no key
        ti = tarfile.TarInfo("somedir")
        ti.type = tarfile.DIRTYPE
        tf.addfile(ti)
        _add(tf, "e.jpg", b"")                   # empty image member
    tar = buf.getvalue()
    idx = index_any(tar)
    assert idx.keys == ["b", "dir/c", "e"]
    got = [tar[r["img_off"]:r["img_off"] + r["img_len"]] for r in idx.samples]
    assert got == [b"B", b"C2", b""]
    assert [(k, i) for k, i, _ in oracle_samples(tar)] == list(zip(idx.keys, got))


def test_tar_index_truncation_and_bad_headers(index_any):
    tar = make_shard(6, seed=1)
    full = index_any(tar)
    # truncated inside the 4th jpg's data: 3 samples, truncation status
    cut = int(full.samples[3]["img_off"]) + 5
    t = index_any(tar[:cut])
    assert t.status == tario.TAR_TRUNCATED and len(t) == 3
    # corrupt checksum of a later header: iteration stops there (tarfile semantics)
    bad = bytearray(tar)
    h = int(full.samples[2]["img_off"]) - 512
    bad[h + 148:h + 156] = b"0000000\x00"
    t = index_any(bytes(bad))
    assert t.status == tario.TAR_BAD_HEADER and len(t) == 2
    # corrupt first header: error, like tarfile.ReadError
    with pytest.raises(tario._lib.DinoError):
        index_any(b"\x01" * 2048)
    assert len(index_any(b"")) == 0
    assert len(index_any(b"\x00" * 1024)) == 0


def test_extract_jpegs_with_meta_records():
    tar = make_shard(10, seed=2)
    recs = tario.extract_jpegs_with_meta(tar)
    ref = oracle_samples(tar)
    assert [r.key for r in recs] == [k for k, _, _ in ref]
    assert all(bytes(r.jpeg) == img for r, (_, img, _) in zip(recs, ref))
    assert recs[3].metadata == json.loads(ref[3][2])
    kept = tario.extract_jpegs_with_meta(tar, min_quality=0.5)
    assert [r.key for r in kept] == [r.key for r in recs if r.metadata["quality_score"] >= 0.5]
    sh = tario.extract_jpegs_with_meta(tar, shuffle_buffer=8, rng=np.random.default_rng(0), copy=True)
    assert sorted(r.key for r in sh) == [r.key for r in recs] and isinstance(sh[0].jpeg, bytes)
    assert tario.extract_jpegs_with_meta(make_shard(3, with_meta=False))[0].metadata is None


@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_gather_packs_ranges(nthreads):
    rng = np.random.default_rng(nthreads)
    items = [rng.integers(0, 256, int(rng.integers(0, 400_000)), dtype=np.uint8) for _ in range(40)]
    items[5] = items[5][:0]
    dst = torch.empty(sum(i.size for i in items) + 7, dtype=torch.uint8)
    off = tario.gather(items, dst, nthreads)
    assert off[0] == 0 and (np.diff(off) == [i.size for i in items]).all()
    flat = dst.numpy()
    for i, it in enumerate(items):
        assert np.array_equal(flat[off[i]:off[i + 1]], it)
    with pytest.raises(tario._lib.DinoError):
        tario.gather(items, torch.empty(10, dtype=torch.uint8))


def test_shm_cache_format_and_views(tmp_path):
    cache = tario.ShmShardCache(job_id="job", base_dir=tmp_path, max_gb=1.0)
    tar = make_shard(5, seed=4)
    src = tmp_path / "shard-000.tar"
    src.write_bytes(tar)
    cache.prefetch(str(src))                                   # node master loads it (in the background)
    cache.prefetch(str(src))                                   # loading already: not scheduled twice
    assert cache.get(str(src)) == tar                          # waits for the background load
    shm = tmp_path / "job" / hashlib.sha1(str(src).encode()).hexdigest()[:16]
    raw = shm.read_bytes()
    assert struct.unpack_from("QQ", raw) == (len(tar), 0xDEADBEEFCAFEF00D) and raw[16:] == tar
    with cache.get_view(str(src)) as v:
        assert bytes(v) == tar
    arr = cache.get_array(str(src))
    assert arr.tobytes() == tar and len(tario.index_tar(arr)) == 5
    assert cache.get(str(src)) == tar and 0 < cache.utilisation < 1
    # a reader that is not the node master waits for the master's write and times out on a
    # missing shard; a corrupt magic is "not ready" (reference _is_ready / _inotify_wait)
    other = tario.ShmShardCache(job_id="job", base_dir=tmp_path, node_master=False, shard_timeout_s=0.2)
    with pytest.raises(TimeoutError, match="waiting for shard"):
        other.get(str(tmp_path / "missing.tar"))
    bad = tmp_path / "job" / hashlib.sha1(b"bad").hexdigest()[:16]
    bad.write_bytes(struct.pack("QQ", 3, 0xDEADBEEFCAFEF00D - 1) + b"abc")
    with pytest.raises(TimeoutError):
        other.get("bad")                                        # not ready: the magic is the ready flag
    assert other.get(str(src)) == tar                           # written by the master: no wait
    cache.close(remove=True)
    assert not shm.exists()


def test_shm_cache_evicts_lru_over_budget(tmp_path):
    tar = make_shard(4, seed=5)
    cache = tario.ShmShardCache(job_id="j2", base_dir=tmp_path, max_gb=2.5 * len(tar) / (1 << 30))
    for k in range(4):
        cache.put(f"s{k}", tar)
    alive = [tario.is_ready(tario.shm_path(cache.base, f"s{k}")) for k in range(4)]
    assert alive == [False, False, True, True]
    cache.close(remove=True)


@pytest.mark.parametrize("world", [1, 2])
def test_batch_feeder_partitions_and_drops_last(tmp_path, world):
    shards = [make_shard(n, seed=10 + k) for k, n in enumerate([7, 5, 9, 4])]
    cache = tario.ShmShardCache(job_id=f"feed{world}", base_dir=tmp_path)
    paths = []
    for k, t in enumerate(shards):
        paths.append(f"/data/shard-{k:03d}.tar")
        cache.put(paths[-1], t)
    for rank in range(world):
        mine = [k for k in range(4) if k % world == rank]              # hpc_source.py:154-156
        expect = [img for k in mine for _, img, _ in oracle_samples(shards[k])]
        feeder = tario.ShardBatchFeeder(cache, paths, batch_size=3, rank=rank, world=world, nthreads=2)
        dst = torch.empty(1 << 16, dtype=torch.uint8)
        got = []
        while True:
            try:
                off = feeder.next_into(dst)
            except StopIteration:
                break
            assert len(off) == 4
            got += [dst.numpy()[off[i]:off[i + 1]].tobytes() for i in range(3)]
        assert got == expect[:len(expect) // 3 * 3]
    cache.close(remove=True)


def _set_header(tar: bytearray, h: int, size_field: bytes) -> None:
    """Overwrite member header h's size field and fix its checksum."""
    tar[h + 124:h + 136] = size_field
    tar[h + 148:h + 156] = b" " * 8
    tar[h + 148:h + 156] = b"%06o\x00 " % sum(tar[h:h + 512])


def test_tar_index_forged_sizes_do_not_overflow():
    """A base-256 or octal size near 2^63 (or a pax size) must not wrap the bounds check
    (data + size > len overflowed): the member is reported truncated and the
    samples before it are kept."""
    tar = make_shard(4, seed=2)
    full = tario.index_tar(tar)
    h = int(full.samples[2]["img_off"]) - 512
    for field in (b"\x80" + b"\x7f" + b"\xff" * 10,          # base-256, ~2^87: rejected
                  b"\x80\x00\x00\x00" + b"\x7f" + b"\xff" * 7,  # base-256, ~2^63 - 1
                  b"\xff" * 12,                              # negative base-256
                  b"7777777777777777"[:11] + b"\x00"):      # octal, 8^11 - 1: fits, truncated
        bad = bytearray(tar)
        _set_header(bad, h, field)
        t = tario.index_tar(bytes(bad))
        assert t.status in (tario.TAR_TRUNCATED, tario.TAR_BAD_HEADER) and len(t) == 2, field
        for r in t.samples:
            assert 0 <= r["img_off"] and r["img_off"] + r["img_len"] <= len(bad)


def test_batch_spans_cover_the_batch_where_it_lies(tmp_path):
    """next_batch_spans: the parts (contiguous shard ranges, tar headers and sidecars included)
    concatenated and cut at offsets/lens give the same images as the packed feed, across shard
    boundaries; retire() balances the bookkeeping; probe_spans == probe of the packed batch."""
    import ctypes

    from dataloader_amd import fallback
    shards = [make_shard(n, seed=20 + k) for k, n in enumerate([7, 5, 9])]
    cache = tario.ShmShardCache(job_id="spans", base_dir=tmp_path)
    paths = []
    for k, t in enumerate(shards):
        paths.append(f"/data/shard-{k:03d}.tar")
        cache.put(paths[-1], t)
    expect = [img for t in shards for _, img, _ in oracle_samples(t)]
    feeder = tario.ShardBatchFeeder(cache, paths, batch_size=4, nthreads=2, register=False)
    got, n_parts = [], []
    while True:
        try:
            bs = feeder.next_batch_spans()
        except StopIteration:
            break
        assert not bs.registered and len(bs.offsets) == 5 and bs.offsets[-1] == sum(n for _, n in bs.parts)
        flat = b"".join(ctypes.string_at(a, n) for a, n in bs.parts)
        imgs = [flat[bs.offsets[i]:bs.offsets[i] + bs.lens[i]] for i in range(4)]
        assert imgs == [ctypes.string_at(int(p), int(n)) for p, n in zip(bs.ptrs, bs.lens)]
        got += imgs
        n_parts.append(len(bs.parts))
        info_s, ws_s, _ = fallback.probe_spans(bs.ptrs, bs.lens, 0)
        dst = torch.empty(1 << 16, dtype=torch.uint8)
        off = tario.gather(list(zip(bs.ptrs.tolist(), bs.lens.tolist())), dst, 1)
        info_p, ws_p, _ = fallback.probe(dst.data_ptr(), off, 4, 0)
        assert np.array_equal(info_s, info_p) and ws_s == ws_p
        for nt in (1, 3):  # the fused pack + probe pass: same bytes, same probe
            dst2 = torch.zeros(1 << 16, dtype=torch.uint8)
            off2, info_g, ws_g, _ = fallback.gather_probe(bs.ptrs, bs.lens, dst2, nt, 0)
            assert np.array_equal(off2, off) and np.array_equal(info_g, info_p) and ws_g == ws_p
            assert torch.equal(dst2[:off[-1]], dst[:off[-1]])
        feeder.retire(bs, None)
    assert got == expect[:len(expect) // 4 * 4] and max(n_parts) == 2   # batches straddle shards
    feeder.close()
    cache.close(remove=True)


@pytest.mark.parametrize("nthreads", [1, 3])
def test_native_feed_batches_epochs_and_errors(tmp_path, nthreads):
    """NativeShardFeed (C++ opener + packer threads; host-only slots without a GPU): the same
    batches as the Python feeder (rank partition, batches straddling shards, last partial batch
    dropped), each probed like dino_probe on the packed bytes; reset starts a new epoch; a
    corrupt shard-cache file is skipped with a warning (reference hpc_source.py:358-366)."""
    import ctypes

    from dataloader_amd import fallback
    shards = [make_shard(n, seed=30 + k) for k, n in enumerate([7, 5, 9, 6, 8])]
    cache = tario.ShmShardCache(job_id=f"nfeed{nthreads}", base_dir=tmp_path)
    paths = []
    for k, t in enumerate(shards):
        paths.append(f"/data/shard-{k:03d}.tar")
        cache.put(paths[-1], t)
    for world in (1, 2):
        for rank in range(world):
            mine = [k for k in range(5) if k % world == rank]
            expect = [img for k in mine for _, img, _ in oracle_samples(shards[k])]
            feed = tario.NativeShardFeed(cache, paths, 4, rank=rank, world=world, nthreads=nthreads, slots=3)
            for epoch in range(2):
                got = []
                while True:
                    try:
                        fb = feed.next_prepared(timeout=10.0)
                    except StopIteration:
                        break
                    assert fb is not None
                    imgs = fb.jpegs()
                    dst = torch.empty(1 << 16, dtype=torch.uint8)
                    off = tario.gather(imgs, dst, 1)
                    info, ws, _ = fallback.probe(dst.data_ptr(), off, 4, 0)
                    assert np.array_equal(fb.offsets, off) and np.array_equal(fb.info, info) and fb.ws == ws
                    got += imgs
                    feed.release(fb)
                assert got == expect[:len(expect) // 4 * 4], (world, rank, epoch)
                feed.reset()
            st = feed.stats()
            assert st["batches"] >= 2 * (len(expect) // 4) and st["shards_failed"] == 0
            feed.close()
    # a shard whose cache file lost its ready magic is skipped, once, with a warning
    bad = tario.shm_path(cache.base, paths[1])
    raw = bytearray(bad.read_bytes())
    raw[8:16] = b"\x00" * 8
    bad.write_bytes(bytes(raw))
    cache._ensure = lambda p: tario.shm_path(cache.base, p)  # the reader trusts the file as it is
    feed = tario.NativeShardFeed(cache, paths, 4, nthreads=nthreads)
    n = 0
    with pytest.warns(RuntimeWarning, match="skipped a shard"):
        while True:
            try:
                fb = feed.next_prepared(timeout=10.0)
            except StopIteration:
                break
            n += 1
            feed.release(fb)
    assert n == (7 + 9 + 6 + 8) // 4 and feed.shard_errors and feed.stats()["shards_failed"] == 1
    feed.close()
    cache.close(remove=True)


def _feed_reader(base, job, paths, rank, world, timeout_s, q, via_backend=False):
    """A non-master rank (spawned process): drive NativeShardFeed over the node cache while the
    master is still writing it; report the bytes of every batch.  ``via_backend``: the cache comes
    from the drop-in factory, MI355XBackend.build_shard_cache (reference dali_backend.py:85-105)."""
    from dataloader_amd import tario as t
    if via_backend:
        from dataloader_amd.backend import MI355XBackend
        cache = MI355XBackend().build_shard_cache(job_id=job, node_master=False, max_gb=1.0, prefetch_window=4,
                                                  timeout_s=timeout_s, warn_threshold=0.85, base_dir=base)
    else:
        cache = t.ShmShardCache(job_id=job, base_dir=base, node_master=False, shard_timeout_s=timeout_s)
    feed = t.NativeShardFeed(cache, paths, 4, rank=rank, world=world, nthreads=2, slots=3)
    out = []
    try:
        while True:
            try:
                fb = feed.next_prepared(timeout=60.0)
            except StopIteration:
                break
            if fb is None:
                out = "stalled"
                break
            out.append(b"".join(fb.jpegs()))
            feed.release(fb)
        q.put((rank, out, list(feed.shard_errors)))
    finally:
        feed.close()
        cache.close()


def _expected_batches(tmp_path, shards, paths, rank, world):
    """Batches of a pre-written cache (the master's view), the bar for the waiting readers."""
    cache = tario.ShmShardCache(job_id="prewritten", base_dir=tmp_path)
    for p, t in zip(paths, shards):
        cache.put(p, t)
    feed = tario.NativeShardFeed(cache, paths, 4, rank=rank, world=world, nthreads=2, slots=3)
    out = []
    while True:
        try:
            fb = feed.next_prepared(timeout=10.0)
        except StopIteration:
            break
        out.append(b"".join(fb.jpegs()))
        feed.release(fb)
    feed.close()
    cache.close(remove=True)
    return out


def test_non_master_ranks_wait_for_the_node_master(tmp_path):
    """Row f2 (reference shard_cache.py:588-603, :373-449, master = local rank 0, loader.py:467):
    two non-master processes drive the native feed over a node cache that the master (this
    process) writes shard by shard with a delay; each gets every batch bit-identical to a
    pre-written cache.  A shard the master never writes times out and is skipped with a warning
    (hpc_source.py:358-366)."""
    import multiprocessing as mp
    import time
    shards = [make_shard(n, seed=60 + k) for k, n in enumerate([9, 6, 8, 7])]
    paths = [f"/lustre/ds/shard-{k:03d}.tar" for k in range(4)]
    expect = {r: _expected_batches(tmp_path, shards, paths, r, 2) for r in range(2)}
    master = tario.ShmShardCache(job_id="live", base_dir=tmp_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_feed_reader, args=(tmp_path, "live", paths, r, 2, 60.0, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    try:
        time.sleep(1.0)                                  # readers are up and waiting on the first shards
        for p, t in zip(paths, shards):
            master.put(p, t)
            time.sleep(0.3)
        got = {}
        for _ in procs:
            r, batches, errs = q.get(timeout=120)
            got[r] = (batches, errs)
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
    for r in range(2):
        batches, errs = got[r]
        assert errs == [] and batches == expect[r] and len(batches) > 0, r
    # a shard the master never writes: the waiting reader times out on it, skips it, goes on
    reader = tario.ShmShardCache(job_id="live", base_dir=tmp_path, node_master=False, shard_timeout_s=0.5)
    feed = tario.NativeShardFeed(reader, paths[:2] + ["/lustre/ds/never.tar"] + paths[2:], 4, nthreads=2)
    n = 0
    with pytest.warns(RuntimeWarning, match="Timed out"):
        while True:
            try:
                fb = feed.next_prepared(timeout=30.0)
            except StopIteration:
                break
            n += 1
            feed.release(fb)
    assert n == sum(len(oracle_samples(t)) for t in shards) // 4 and len(feed.shard_errors) == 1
    feed.close()
    with pytest.raises(TimeoutError):
        with reader.get_view("/lustre/ds/never.tar"):
            pass
    master.close(remove=True)


def test_backend_shard_cache_master_and_readers(tmp_path):
    """the drop-in factory gives the node-shared cache.  One master (this process,
    ``build_shard_cache(node_master=True)``) loads the shards from the filesystem in the
    background (``prefetch``); two non-master processes (``node_master=False``) drive the native
    feed over it while it is being written; each gets every batch bit-identical to a pre-written
    cache."""
    import multiprocessing as mp

    from dataloader_amd.backend import MI355XBackend
    shards = [make_shard(n, seed=90 + k) for k, n in enumerate([9, 6, 8, 7, 5])]
    src_dir = tmp_path / "lustre"
    src_dir.mkdir()
    paths = []
    for k, t in enumerate(shards):
        p = src_dir / f"shard-{k:03d}.tar"
        p.write_bytes(t)
        paths.append(str(p))
    expect = {r: _expected_batches(tmp_path, shards, paths, r, 2) for r in range(2)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_feed_reader, args=(tmp_path, "nodejob", paths, r, 2, 60.0, q, True))
             for r in range(2)]
    for pr in procs:
        pr.start()
    master = None
    try:
        import time
        time.sleep(1.0)                                  # readers up and waiting before the master exists
        master = MI355XBackend().build_shard_cache(job_id="nodejob", node_master=True, max_gb=1.0,
                                                   prefetch_window=2, timeout_s=60.0, warn_threshold=0.85,
                                                   base_dir=tmp_path)
        for p in paths:
            master.prefetch(p)
        got = {}
        for _ in procs:
            r, batches, errs = q.get(timeout=120)
            got[r] = (batches, errs)
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
    for r in range(2):
        batches, errs = got[r]
        assert errs == [] and batches == expect[r] and len(batches) > 0, r
    for p, t in zip(paths, shards):                      # the master's own view of its cache
        assert master.get(p) == t
    master.close(remove=True)


def test_native_feed_shuffle_orders(tmp_path):
    """shuffle=True: the reference's per-epoch shard order (numpy default_rng(seed + rank +
    epoch * 997).shuffle, hpc_source.py:263, 488-500) and a seeded in-shard order; the same
    samples per epoch, a different order per epoch, the same order for the same (seed, epoch)."""
    shards = [make_shard(n, seed=80 + k) for k, n in enumerate([8, 8, 8, 8, 8])]
    cache = tario.ShmShardCache(job_id="shuf", base_dir=tmp_path)
    paths = [f"/d/s{k}.tar" for k in range(5)]
    for p, t in zip(paths, shards):
        cache.put(p, t)

    def epoch_imgs(feed):
        got = []
        while True:
            try:
                fb = feed.next_prepared(timeout=10.0)
            except StopIteration:
                break
            got += fb.jpegs()
            feed.release(fb)
        return got

    f1 = tario.NativeShardFeed(cache, paths, 4, nthreads=2, shuffle=True, seed=5)
    f2 = tario.NativeShardFeed(cache, paths, 4, nthreads=2, shuffle=True, seed=5)
    order = list(paths)
    np.random.default_rng(5).shuffle(order)
    assert f1.epoch_order() == order
    e0 = epoch_imgs(f1)
    f1.reset()
    e1 = epoch_imgs(f1)
    assert e0 == epoch_imgs(f2)                          # deterministic
    allimgs = sorted(img for t in shards for _, img, _ in oracle_samples(t))
    assert sorted(e0) == sorted(e1) == allimgs and e0 != e1
    plain = [img for p in order for _, img, _ in oracle_samples(shards[paths.index(p)])]
    assert e0 != plain                                   # samples shuffled inside each shard
    first = {img for _, img, _ in oracle_samples(shards[paths.index(order[0])])}
    assert set(e0[:8]) == first                          # ... but shard by shard
    # resume: a fresh feed reset to epoch 2 gives the epoch-2 order of a feed that ran
    # epochs 0 and 1, shard order and in-shard order alike
    f1.reset()
    e2 = epoch_imgs(f1)
    f3 = tario.NativeShardFeed(cache, paths, 4, nthreads=2, shuffle=True, seed=5)
    f3.reset(epoch=2)
    assert f3.epoch_order() == f1.epoch_order() and epoch_imgs(f3) == e2 != e1
    for f in (f1, f2, f3):
        f.close()
    cache.close(remove=True)
