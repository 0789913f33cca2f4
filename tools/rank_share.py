#!/usr/bin/env python3
"""Strong-scaling rehearsal on ONE GPU: render each rank's share of the frame
alone (row-cyclic tiles of rank r of N) and time it with HIP events.  The
slowest rank bounds an N-GPU frame, so T(1) / max_r T(r of N) is the kernel
part of the N-GPU speed-up (the gather comes on top).

    python tools/rank_share.py --scene csg32 --worlds 1 2 4 8
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="csg32")
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tile-rows", type=int, default=4)
    ap.add_argument("--tracer", default="auto")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--stream-frames", type=int, default=0,
                    help="also time this many back-to-back frames of each share alternating over two streams "
                         "(frames in flight: a frame's first tiles start while the previous frame's last finish)")
    args = ap.parse_args()

    import torch
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl

    torch.cuda.set_device(0)
    r = wl.Renderer("share", max_nodes=4096)
    info = scenes.build(args.scene, r)
    over = {}
    if args.width:
        over["width"] = args.width
    if args.height:
        over["height"] = args.height
    if args.spp:
        over["spp"] = args.spp
    p = info.params(**over)
    r.set_tracer(args.tracer)
    W, H, T = p.width, p.height, args.tile_rows
    out = torch.empty((wl.local_rows(H, T, 1), W, 4), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    r.render_rows_device(p, out.data_ptr(), T, 0, 1, s.cuda_stream)  # warm-up (JIT)
    torch.cuda.synchronize()
    res = {"scene": args.scene, "size": f"{W}x{H}x{p.spp}", "path": r.trace_path(), "worlds": {}}
    t1 = None
    for n in args.worlds:
        per_rank = []
        for rank in range(n):
            ms = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                r.render_rows_device(p, out.data_ptr(), T, rank, n, s.cuda_stream)
                b.record(s)
                b.synchronize()
                ms.append(a.elapsed_time(b))
            if args.stream_frames:
                ss = [torch.cuda.Stream(), torch.cuda.Stream()]
                outs = [out, torch.empty_like(out)]
                for k in range(2):  # first use of each stream and buffer, untimed
                    r.render_rows_device(p, outs[k].data_ptr(), T, rank, n, ss[k].cuda_stream)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for st in ss:
                    st.wait_event(a)
                for k in range(args.stream_frames):
                    r.render_rows_device(p, outs[k & 1].data_ptr(), T, rank, n, ss[k & 1].cuda_stream)
                for st in ss:
                    s.wait_stream(st)
                b.record(s)
                b.synchronize()
                ms = [a.elapsed_time(b) / args.stream_frames]  # per frame, overlapped
            per_rank.append(min(ms))
        worst = max(per_rank)
        if n == 1:
            t1 = worst
        res["worlds"][n] = {"rank_ms": [round(x, 3) for x in per_rank], "max_ms": round(worst, 3),
                            "speedup_kernel": round(t1 / worst, 3) if t1 else None}
        print(f"[share] N={n} max {worst:.3f} ms ranks {['%.3f' % x for x in per_rank]}"
              + (f" speed-up {t1 / worst:.2f}" if t1 else ""), flush=True)
    print(json.dumps(res))
    r.close()


if __name__ == "__main__":
    main()
