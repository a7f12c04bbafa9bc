"""bench.py's roofline accounting: a kernel launched once per view class
is charged all its launches of a step, the dominant kernel's fraction recomputes by hand from
bytes per step and its time per step, and the line carries the traffic / interface ratio and
the path fraction.  CPU only (synthetic per-kernel times)."""

from __future__ import annotations

import bench


def _leg(steps):
    # k_hresize: 2 launches per step of 1.1 ms each; k_huff1: 1 launch of 0.9 ms
    return {"dt": steps * 3.0e-3, "t_ser": None,
            "ktimes": {"k_hresize": (2 * 1.1 * steps, 2 * steps), "k_huff1": (0.9 * steps, steps)}}


def test_per_step_charging_of_per_class_kernels(monkeypatch):
    monkeypatch.setattr(bench, "load_traffic", lambda tag: ({"k_hresize": 3.0e8, "k_huff1": 5.0e8}, "r99_pmc_c3.json"))
    steps, B = 10, 512
    ab = {"path": 1.0e6, "s_jpeg": 8.0e4, "pixels": 3.0e5, "k_hresize": 2.0e6, "k_huff1": 9.0e4}
    out = bench.summarize(_leg(steps), ab, B, steps, 1, "c3")
    rf = out["roofline"]
    assert rf["kernel"] == "k_hresize"                      # 2.2 ms per step beats 0.9
    assert rf["launches_per_step"] == 2.0
    assert abs(rf["kernel_ms_per_step"] - 2.2) < 1e-9
    # bytes of a step over the kernel's time per step (not over one launch)
    assert abs(rf["achieved"] - round(1.0e6 * B / 2.2e-3 / 1e9, 2)) < 1e-6
    assert abs(rf["frac"] - round(1.0e6 * B / 2.2e-3 / 1e9 / 8000.0, 5)) < 1e-9
    # per launch: half the step's bytes over the mean launch time -> the same ratio
    assert rf["algorithmic_bytes_per_launch"] == int(1.0e6 * B / 2)
    assert abs(rf["algorithmic_bytes_per_launch"] / (rf["avg_launch_ms"] * 1e-3) / 1e9 - rf["achieved"]) < 0.05
    # traffic per launch over the kernel's own interface bytes per launch
    assert abs(rf["traffic_over_interface"] - round(3.0e8 / (2.0e6 * B / 2), 3)) < 1e-9
    assert rf["path_frac"] == out["path_roofline"]["frac"]
    assert abs(rf["path_frac"] - round(1.0e6 * B / 3.0e-3 / 1e9 / 8000.0, 5)) < 1e-9
    hr = out["roofline_kernels"]["k_hresize"]
    assert hr["interface_bytes_per_step"] == int(2.0e6 * B) and hr["interface_bytes_per_launch"] == int(1.0e6 * B)
    assert abs(hr["frac"] - round(2.0e6 * B / 2.2e-3 / 1e9 / 8000.0, 4)) < 1e-9
