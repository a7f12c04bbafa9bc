"""Progressive routing through the product iterator (host JPEG feed, depth 3): images/s
for batches of B 640x480 JPEGs of which k are progressive, per ``multiscan_route``.
Writes one JSON line per (k, route) to stdout."""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from bench import make_unique  # noqa: E402
from dataloader_amd.config import DINOAugConfig  # noqa: E402
from dataloader_amd.pipeline import MI355XAugPipeline, MI355XPipelineIterator  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--batches", type=int, default=24)
    ap.add_argument("--ks", default="0,1,4,16,64")
    ap.add_argument("--routes", default="device,auto,host,side")
    ap.add_argument("--side-ahead", type=int, default=24)
    ap.add_argument("--warm", type=int, default=3, help="batches before the timed region")
    ap.add_argument("--repeat", type=int, default=1, help="runs of each (k, route) in this process")
    ap.add_argument("--backend", action="store_true",
                    help="build through MI355XBackend.build_pipeline + build_pipeline_iterator (as bench's c2_prog)")
    args = ap.parse_args()
    B = args.batch
    base = make_unique(B, 640, 480, 1, False, 8)
    prog = make_unique(64, 640, 480, 2, False, 8, prog_frac=1.0)
    cfg = DINOAugConfig()
    for k in [int(x) for x in args.ks.split(",")]:
        # the k progressive images spread over the batch, a different set each batch
        batches = []
        for b in range(args.batches):
            j = list(base)
            for t in range(k):
                j[(t * B) // max(k, 1) + b % max(1, B // max(k, 1))] = prog[(b * k + t) % len(prog)]
            batches.append(j)
        for route in [r for r in args.routes.split(",") for _ in range(args.repeat)]:
            if k == 0 and route not in ("auto", "side"):
                continue
            src = iter(batches)
            if args.backend:
                from dataloader_amd.backend import MI355XBackend
                from dataloader_amd.config import DinoV2AugSpec, PipelineConfig

                class _Src:
                    _batch_size, _resolution_src = B, None

                    def __call__(self):
                        return next(src)
                spec = DinoV2AugSpec(aug_cfg=cfg)
                be = MI355XBackend(multiscan_route=route)
                pipe = be.build_pipeline(_Src(), spec, PipelineConfig(device_id=0, seed=1, gpu_queue=6), None)
                it = be.build_pipeline_iterator(pipe, spec, spec.output_map, B)
            else:
                pipe = MI355XAugPipeline(lambda: next(src), cfg, B, seed=1, depth=3, multiscan_route=route,
                                         side_ahead=args.side_ahead)
                it = MI355XPipelineIterator(pipe, [f"view_{i}" for i in range(cfg.n_views)], B)
            n = 0
            t0 = None
            for i, _ in enumerate(it):
                if i == args.warm:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                elif i > args.warm:
                    n += B
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            hs = {k: round(v * 1e3 / max(1, args.batches), 3) for k, v in pipe.host_seconds.items()}
            side = getattr(pipe, "_side", None)
            stats = pipe.flush_stats()
            pipe.close()
            print(json.dumps({"k_progressive": k, "route": route, "batch": B, "images_per_s": round(n / dt, 1),
                              "host_decoded": stats["host_decoded"], "side_decoded": stats.get("side_decoded"), "side_urgent": stats.get("side_urgent"),
                              "batches": args.batches, "warm": args.warm, "side_ahead": args.side_ahead,
                              "host_ms_per_batch": hs,
                              "side_launches": getattr(side, "launches", None),
                              "side_phase_ms_per_batch": {k: round(v * 1e3 / args.batches, 3) for k, v in side.phase_seconds.items()} if side else None,
                              "side_host_ms_per_batch": round(side.host_seconds * 1e3 / args.batches, 3) if side else None,
                              "status": dict(stats["status"])}), flush=True)


if __name__ == "__main__":
    main()
