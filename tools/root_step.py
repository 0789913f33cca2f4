#!/usr/bin/env python3
"""Rank 0's whole per-frame step of an N-GPU frame, timed on ONE GPU (VERDICT r2
item 2), next to every other rank's share.

An N-GPU frame (bench.py's RCCL path, or wo_renderer_set_devices' peer-DMA path) costs
rank 0 more than its share of the render: it also receives N-1 shares, un-interleaves
the frame (assemble_kernel) and, for a presented frame, encodes it (srgb8_kernel).  Per
frame, on rank 0's GPU:

    render stream:   rank 0's share -> its slice of the gather buffer
    copy stream:     after the render, N-1 device copies of a share's bytes into the
                     other slices (stands in for the incoming peer DMA; a local copy
                     reads and writes this HBM, the real transfer only writes it:
                     conservative)
    assemble stream: after the copies, assemble_kernel into the frame + the sRGB
                     encode (with --no-encode: the bench's frame, which is not
                     presented)
    map-back stream: after the encode, the present encode's D2H into pinned host
                     memory (--map-back bgra, draw_frame's default; `float` adds the
                     float frame, `none` skips it) -- wo_renderer_draw_frame's copy
                     stream

two frames in flight (two gather buffers, two render streams), F frames back to back.
Every other rank's step is its share alone, timed the same way (back to back over two
streams).  Projected N-GPU frame time = max(rank 0's step, the slowest other share);
speed-up = one GPU's frame time (the N = 1 bench's way: back to back, one stream) over
it.

    python tools/root_step.py --scene csg32 --worlds 2 4 8
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
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--no-encode", action="store_true")
    ap.add_argument("--tile-rows", type=int, default=4, help="rows per row-cyclic band (bench.py --tile-rows)")
    ap.add_argument("--share-streams", type=int, default=2, choices=[1, 2],
                    help="render streams the other ranks' shares alternate over (2: as rank 0's frames)")
    ap.add_argument("--band", default="auto",
                    help="row-band weighting CYCLE:SKIP (rank 0 sits out SKIP of every CYCLE rounds), 'auto' = "
                         "wololo.default_band(N) as bench.py uses it, '0:0' = a band per rank and round")
    ap.add_argument("--streams", default="bench", choices=["bench", "null", "split"],
                    help="rank 0's streams: 'bench' = bench.py's two render streams + one created stream "
                         "for the copies, assemble, encode and D2H; 'null' = the same on the default stream "
                         "(bench.py before round 5: its kernels leave the two render streams on one hardware "
                         "queue, so consecutive frames stop overlapping); 'split' = separate copy / assemble / "
                         "D2H streams (rounds 3-5)")
    ap.add_argument("--map-back", default="bgra", choices=["split", "bgra", "direct", "float", "none"],
                    help="the presented frame's D2H: 'bgra' = rank 0 encodes and copies the whole frame after "
                         "the assembly (draw_frame's default); 'split' = every rank encodes its own rows and "
                         "copies them to the host (WOLOLO_PRESENT_SPLIT=1); 'float' adds the float frame; "
                         "'direct' = the encode kernel writes the pinned host frame itself (no copy); 'none' skips it")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process, as bench.py sets it at N > 1 (0: leave it)")
    args = ap.parse_args()
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 16))

    import torch
    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl

    torch.cuda.set_device(0)
    r = wl.Renderer("root-step", max_nodes=4096)
    info = scenes.build(args.scene, r)
    over = {k: getattr(args, k) for k in ("width", "height", "spp") if getattr(args, k)}
    p = info.params(**over)
    W, H, T, F = p.width, p.height, args.tile_rows, args.frames
    main_s = torch.cuda.current_stream()

    def timed(fn):
        best = None
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record(main_s)
            fn(a)
            b.record(main_s)
            b.synchronize()
            ms = a.elapsed_time(b) / F
            best = ms if best is None else min(best, ms)
        return best

    # one GPU, the whole frame back to back on one stream (bench.py N = 1)
    full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    r.render_rows_device(p, full.data_ptr(), T, 0, 1, main_s.cuda_stream)  # warm-up (JIT)
    torch.cuda.synchronize()

    def one_gpu(start):
        for _ in range(F):
            r.render_rows_device(p, full.data_ptr(), T, 0, 1, main_s.cuda_stream)

    t1 = timed(one_gpu)
    print(f"[root] N=1 {t1:.3f} ms per frame", flush=True)
    # this box's pinned D2H rate at the whole present frame and at one rank's share of it
    d2h = {}
    for mb_bytes in (W * H * 4, W * H * 4 // 8):
        dsrc = torch.empty(mb_bytes // 4, dtype=torch.int32, device="cuda")
        hdst = torch.empty(mb_bytes // 4, dtype=torch.int32).pin_memory()
        hdst.copy_(dsrc, non_blocking=True)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main_s)
        for _ in range(20):
            hdst.copy_(dsrc, non_blocking=True)
        b.record(main_s)
        b.synchronize()
        ms = a.elapsed_time(b) / 20
        d2h[mb_bytes] = (ms, mb_bytes / ms / 1e6)
    print("[root] pinned D2H: " + ", ".join(f"{k / 1e6:.2f} MB {v[0] * 1e3:.0f} us ({v[1]:.1f} GB/s)"
                                           for k, v in d2h.items()), flush=True)
    res = {"scene": args.scene, "size": f"{W}x{H}x{p.spp}", "path": r.trace_path(), "one_gpu_ms": round(t1, 4),
           "d2h_gbps": {str(k): round(v[1], 2) for k, v in d2h.items()},
           "encode": not args.no_encode, "map_back": "none" if args.no_encode else args.map_back, "worlds": {}}
    split = not args.no_encode and args.map_back == "split"
    direct = not args.no_encode and args.map_back == "direct"
    mapback = not args.no_encode and args.map_back not in ("none", "split")
    hb = [torch.empty((H, W), dtype=torch.int32).pin_memory() for _ in range(2)] if mapback else []
    hf = [torch.empty((H, W, 4), dtype=torch.float32).pin_memory() for _ in range(2)] \
        if mapback and args.map_back == "float" else []
    for n in args.worlds:
        band = wl.default_band(n) if args.band == "auto" else tuple(int(x) for x in args.band.split(":"))
        r.set_band_weight(*band)
        lr = wl.local_rows(H, T, n, band)
        share_bytes = lr * W * 16
        rs = [torch.cuda.Stream(), torch.cuda.Stream()]
        if args.streams == "null":
            cps = asm = d2h = main_s
        elif args.streams == "bench":
            cps = asm = d2h = torch.cuda.Stream()
        else:
            cps, asm, d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
        gather = [torch.empty((n, lr, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
        frames = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
        bgra = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(2)]
        src = torch.zeros((lr, W, 4), dtype=torch.float32, device="cuda")
        # the split present: a rank's rows encoded (device) and copied to pinned host memory
        # on its own stream after its render (the library's copy stream)
        pst = [torch.cuda.Stream(), torch.cuda.Stream()] if split else []
        pdev = [torch.empty((lr, W), dtype=torch.int32, device="cuda") for _ in range(2)] if split else []
        phost = [torch.empty((lr, W), dtype=torch.int32).pin_memory() for _ in range(2)] if split else []

        def present_rows(b, rows, st_render):
            # encode + D2H of one rank's rows (1/n of the frame); returns the encode-done event
            ev = torch.cuda.Event()
            ev.record(st_render)
            pst[b].wait_event(ev)
            wl.srgb8_encode_device(rows.data_ptr(), pdev[b].data_ptr(), lr * W, pst[b].cuda_stream)
            enc = torch.cuda.Event()
            enc.record(pst[b])
            with torch.cuda.stream(pst[b]):
                phost[b].copy_(pdev[b], non_blocking=True)
            return enc

        def share(rank):
            def go(start):
                for st in rs:
                    st.wait_event(start)
                for st in pst:
                    st.wait_event(start)
                enc = [None, None]
                for k in range(F):
                    st = rs[k & 1] if args.share_streams == 2 else rs[0]
                    if enc[k & 1] is not None:  # the share buffer is free once its encode has read it
                        st.wait_event(enc[k & 1])
                    r.render_rows_device(p, gather[k & 1][0].data_ptr(), T, rank, n, st.cuda_stream)
                    if split:
                        enc[k & 1] = present_rows(k & 1, gather[k & 1][0], st)
                for st in rs + pst:
                    main_s.wait_stream(st)
            return go

        def root(start):
            for st in rs + [cps, asm, d2h] + pst:
                st.wait_event(start)
            released = [None, None]
            mapped = [None, None]  # the D2H that last read the slot's encode / frame
            for k in range(F):
                b = k & 1
                if released[b] is not None:
                    rs[b].wait_event(released[b])
                r.render_rows_device(p, gather[b][0].data_ptr(), T, 0, n, rs[b].cuda_stream)
                enc = present_rows(b, gather[b][0], rs[b]) if split else None
                done = torch.cuda.Event()
                done.record(rs[b])
                cps.wait_event(done)
                with torch.cuda.stream(cps):
                    for i in range(1, n):
                        gather[b][i].copy_(src, non_blocking=True)
                copied = torch.cuda.Event()
                copied.record(cps)
                asm.wait_event(copied)
                if mapped[b] is not None:
                    asm.wait_event(mapped[b])
                wl.assemble_rows_device(gather[b].data_ptr(), frames[b].data_ptr(), W, H, T, n, asm.cuda_stream,
                                        band)
                if not args.no_encode and not split:
                    # 'direct': the encode's stores go to the pinned host frame (device-visible)
                    wl.srgb8_encode_device(frames[b].data_ptr(), (hb[b] if direct else bgra[b]).data_ptr(), W * H,
                                           asm.cuda_stream)
                if enc is not None:  # the gather buffer is free once the split encode has read it too
                    asm.wait_event(enc)
                ev = torch.cuda.Event()
                ev.record(asm)
                released[b] = ev
                if mapback and not direct:
                    d2h.wait_event(ev)
                    with torch.cuda.stream(d2h):
                        hb[b].copy_(bgra[b], non_blocking=True)
                        if hf:
                            hf[b].copy_(frames[b], non_blocking=True)
                    mev = torch.cuda.Event()
                    mev.record(d2h)
                    mapped[b] = mev
            for st in rs + [cps, asm, d2h] + pst:
                main_s.wait_stream(st)

        root(torch.cuda.Event())  # first use of the streams and buffers, untimed
        torch.cuda.synchronize()
        root_ms = timed(root)
        others = [timed(share(k)) for k in range(1, n)]
        worst_other = max(others) if others else 0.0
        proj = max(root_ms, worst_other)
        res["worlds"][n] = {"band": list(band), "root_step_ms": round(root_ms, 4),
                            "other_share_ms": [round(x, 4) for x in others],
                            "share_bytes": share_bytes, "projected_frame_ms": round(proj, 4),
                            "projected_speedup": round(t1 / proj, 3)}
        print(f"[root] N={n} band {band[0]}:{band[1]} rank 0 step {root_ms:.3f} ms (share + {n - 1} copies of {share_bytes / 1e6:.1f} MB "
              f"+ assemble{'' if args.no_encode or split else ' + encode'}{' + D2H ' + args.map_back if mapback else ''}"
              f"{'; every rank: its rows encoded + D2H (split present)' if split else ''}), "
              f"slowest other share {worst_other:.3f} ms "
              f"-> {proj:.3f} ms per frame, {t1 / proj:.2f}x", flush=True)
    print(json.dumps(res))
    r.close()


if __name__ == "__main__":
    main()
