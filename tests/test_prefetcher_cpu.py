"""The pipeline's host-half prefetcher (pipeline._Prefetcher) on CPU: with a list source its
pull runs on a thread of its own and PACK_THREADS threads pack concurrently (round 6);
batches still come out in the source's order, the source's end and its errors (pull or
pack) reach the launch thread in place, and close() frees every prepared batch that was
never handed out."""

from __future__ import annotations

import random
import threading
import time

import pytest

from dataloader_amd import pipeline as P


class _FakePipe:
    """What _Prefetcher calls on its pipeline: _pull_raw, _pack_raw, _stage_early, _drop."""

    def __init__(self, n: int, fail_at: int | None = None, spans: bool = False, pack_fail_at: int | None = None):
        self._spans_feed = spans
        self.pack_fail_at = pack_fail_at
        self.rng = random.Random(7)
        self._native = False
        self.n, self.fail_at = n, fail_at
        self.k = 0
        self.pull_threads, self.pack_threads = set(), set()
        self.dropped, self.staged = [], []
        self.lock = threading.Lock()

    def _pull_raw(self):
        self.pull_threads.add(threading.current_thread().name)
        if self.k == self.fail_at:
            self.k += 1
            raise ValueError("source broke")
        if self.k >= self.n:
            raise StopIteration
        k, self.k = self.k, self.k + 1
        time.sleep(0.001)
        return k

    def _pack_raw(self, raw):
        self.pack_threads.add(threading.current_thread().name)
        time.sleep(0.004 * self.rng.random())  # uneven packs: batches finish out of order
        if raw == self.pack_fail_at:
            raise RuntimeError("pack broke")
        pb = P._Prepared(None, None, None, None, 0, 0, (0, 0), {})
        pb.k = raw
        return pb

    def _prepare_next(self):
        return self._pack_raw(self._pull_raw())

    def _stage_early(self, pb):
        with self.lock:
            self.staged.append(pb.k)

    def _drop(self, pb):
        with self.lock:
            self.dropped.append(pb.k)


def _drain(pf):
    got = []
    while True:
        try:
            got.append(pf.get().k)
        except StopIteration:
            return got


@pytest.mark.parametrize("packers", [1, 2, 3])
def test_list_source_pull_runs_on_its_own_thread_in_order(packers, monkeypatch):
    monkeypatch.setenv("DINO_PACK_THREADS", str(packers))
    pipe = _FakePipe(40)
    pf = P._Prefetcher(pipe, 3)
    try:
        assert _drain(pf) == list(range(40))
        assert pf.finished
    finally:
        pf.close()
    assert pipe.pull_threads == {"dino-pull"}
    assert pipe.pack_threads <= {f"dino-prefetch-{k}" for k in range(packers)} and pipe.pack_threads
    assert sorted(pipe.staged) == list(range(40))


def test_spans_sources_keep_one_thread():
    pipe = _FakePipe(10, spans=True)
    pf = P._Prefetcher(pipe, 2)
    try:
        assert _drain(pf) == list(range(10))
    finally:
        pf.close()
    assert pipe.pull_threads == {"dino-prefetch"} == pipe.pack_threads


@pytest.mark.parametrize("packers", [1, 2])
def test_source_error_reaches_the_launch_thread_after_the_batches_before_it(packers, monkeypatch):
    monkeypatch.setenv("DINO_PACK_THREADS", str(packers))
    pipe = _FakePipe(20, fail_at=7)
    pf = P._Prefetcher(pipe, 2)
    try:
        got = [pf.get().k for _ in range(7)]
        assert got == list(range(7))
        with pytest.raises(ValueError, match="source broke"):
            pf.get()
    finally:
        pf.close()


@pytest.mark.parametrize("packers", [1, 2])
def test_close_drops_prepared_batches_never_handed_out(packers, monkeypatch):
    monkeypatch.setenv("DINO_PACK_THREADS", str(packers))
    pipe = _FakePipe(1000)
    pf = P._Prefetcher(pipe, 4)
    first = pf.get().k
    time.sleep(0.05)  # let the queues fill
    pf.close()
    assert first == 0
    # everything prepared after the first hand-out was either dropped or never made
    assert set(pipe.dropped) <= set(range(1, 1000)) and len(pipe.dropped) >= 1
    assert not any(t.is_alive() for t in pf._threads)


@pytest.mark.parametrize("packers", [1, 2])
def test_pack_error_arrives_in_place(packers, monkeypatch):
    monkeypatch.setenv("DINO_PACK_THREADS", str(packers))
    pipe = _FakePipe(30, pack_fail_at=11)
    pf = P._Prefetcher(pipe, 3)
    try:
        assert [pf.get().k for _ in range(11)] == list(range(11))
        with pytest.raises(RuntimeError, match="pack broke"):
            pf.get()
    finally:
        pf.close()
