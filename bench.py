#!/usr/bin/env python3
"""Headline benchmark: Mrays/s + fps of the CSG path tracer at 1920x1080, 64 spp,
8 bounces on the 32-primitive CSG scene (BASELINE.json metric, config C3), on
1..8 MI355X of one node.

One process per GPU (torchrun).  Every rank renders its row-cyclic tiles of the
SAME frame (strong scaling: the frame is fixed, rows are split), then the tiles
are gathered to rank 0 over RCCL (torch.distributed "nccl") and un-interleaved by
a HIP kernel.  A step = one full frame including the gather.

    python bench.py                       # N=1, defaults finish in about a minute
    torchrun --nproc-per-node 8 bench.py --gpus 8
    python bench.py --gpus 8              # the same: starts torch.distributed.run itself
    python bench.py --gpus 8 --single-process
                                          # one process over 8 GPUs through the C API
                                          # (wo_renderer_set_devices, peer-DMA gather)

--gpus N must match the ranks that actually run: under a launcher WORLD_SIZE must
equal N, and N ranks on the RCCL backend need N visible GPUs; anything else exits
with status 2 (--stack-ranks allows more ranks than GPUs, for rehearsals only).

Prints ONE JSON line on rank 0.  `value` = traced ray segments of the whole frame
(all ranks) / max-over-ranks wall time of the timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/s + fps at 1920x1080x64spp, 32-prim CSG, 1/2/4/8 MI355X"
# /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prewarm-s", type=float, default=0.3,
                    help="untimed frames before the warmup steps until this much wall time has passed (clock ramp)")
    ap.add_argument("--scene", default="csg32",
                    choices=["csg32", "csg32_nested", "csg360_nested", "rtiow_cover", "csg256_balanced", "csg256_chain", "csg512_balanced", "csg32_union", "csg256_balanced_union",
                             "sphere256"])
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--tile-rows", type=int, default=4)
    ap.add_argument("--band", default="auto",
                    help="row-band weighting of an N-rank frame, CYCLE:SKIP: rank 0, which also receives the "
                         "gather and assembles, sits out SKIP of every CYCLE rounds of bands; 'auto' = "
                         "wololo.default_band(N), '0:0' = one band per rank and round")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count-work", action="store_true",
                    help="skip the executed-work counting frame (roofline.achieved then uses the brute-force count)")
    ap.add_argument("--tracer", default=os.environ.get("WOLOLO_TRACER", "auto"),
                    choices=["auto", "interpreter", "jit", "lanes"],
                    help="path-tracer kernel (renderer_ext.h Wo_Tracer); results are identical")
    ap.add_argument("--jit", type=int, default=None, help="legacy: 0 = --tracer interpreter")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo stages the gather through host memory (for rehearsing N>1 ranks on one GPU)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="N>1: GPU_MAX_HW_QUEUES for this rank's process (HIP's default is 4; rank 0's two "
                         "render streams, its gather stream and the default stream then share queues, and a "
                         "render queued behind a gather stops overlapping the previous frame; 0 = leave the "
                         "environment alone)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N>1: gather each frame before the next renders (default: frame k+1 renders while frame k "
                         "is gathered, with either backend)")
    ap.add_argument("--frames-in-flight", type=int, default=None,
                    help="render streams / buffers: frame k+1 may start while frame k's last tiles finish "
                         "(default: 2 for pipelined N>1 runs, whose short per-rank launches lose their tails "
                         "otherwise; 1 at N=1, where the per-launch HIP-event durations feed the roofline)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives all N GPUs through the C API (wo_renderer_set_devices: each rank on its "
                         "own device and stream, peer-DMA gather into rank 0, assembled there); a step is "
                         "wo_renderer_render_frame_device")
    ap.add_argument("--stack-ranks", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share devices): rehearsal only, the line says so")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 checks the assembled frame against a single full-frame render (bit-exact)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-dispatch HBM bytes measured by rocprofv3 --pmc (profiles/*.json) for roofline.traffic")
    ap.add_argument("--side-scenes", default="csg32_nested",
                    help="N=1 csg32 runs only: comma-separated scenes measured after the headline in the same "
                         "invocation and reported as sub-objects of the line ('' = none)")
    ap.add_argument("--no-draw-frame", action="store_true",
                    help="N=1: skip the draw_frame leg (wo_renderer_draw_frame frames, map-back included)")
    ap.add_argument("--draw-frames", type=int, default=60, help="frames of the draw_frame leg")
    return ap.parse_args()


def fail(msg: str, code: int = 2):
    print(f"[bench] error: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


def visible_devices() -> int:
    # counting devices does not initialise HIP on this image (no GPU context yet)
    import torch
    return torch.cuda.device_count()


def self_launch(args) -> int:
    """`bench.py --gpus N` without a launcher: run N ranks under torch.distributed.run
    as a child process (nothing here has touched the GPU) and return its status."""
    ndev = visible_devices()
    if ndev < args.gpus and not args.stack_ranks:
        fail(f"--gpus {args.gpus} needs {args.gpus} GPUs, {ndev} visible (use --stack-ranks to rehearse "
             f"{args.gpus} ranks on fewer, with --dist-backend gloo)")
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] no launcher: starting {args.gpus} ranks with torch.distributed.run", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.single_process:
        if world_env not in (None, "1"):
            fail(f"--single-process drives every GPU from one process; WORLD_SIZE={world_env}")
        return single_process(args)
    if world_env is None and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(world_env or "1")
    if world != args.gpus:
        fail(f"--gpus {args.gpus} but {world} ranks are running (WORLD_SIZE)")
    if world > 1 and args.hw_queues > 0:
        # before the first HIP call of this process (tools/root_step.py, N = 8, rank 0's
        # step: csg32 0.385 -> 0.355 ms, csg32_nested 1.116 -> 0.945 ms with 8 queues)
        # --hw-queues 0 leaves the environment's value alone; otherwise an inherited
        # value is replaced, and said so (the GPU box exports HIP's default, 4; the
        # line records the value used in config.hw_queues)
        want = str(min(args.hw_queues, 16))
        had = os.environ.get("GPU_MAX_HW_QUEUES")
        if had is not None and had != want:
            print(f"[bench] GPU_MAX_HW_QUEUES={had} from the environment replaced by {want} "
                  f"(--hw-queues; 0 keeps it)", file=sys.stderr)
        os.environ["GPU_MAX_HW_QUEUES"] = want
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev < world and not args.stack_ranks:
        fail(f"{world} ranks need {world} GPUs, {ndev} visible (--stack-ranks with --dist-backend gloo "
             f"rehearses them on fewer)")
    if ndev < world and args.dist_backend == "nccl":
        fail("RCCL cannot put two ranks on one GPU: stacked ranks need --dist-backend gloo")
    ranks_stacked = ndev < world
    dev_index = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl

    r = wl.Renderer(f"bench{rank}", max_nodes=4096)
    if args.scene == "sphere256":
        info = scenes.sphere256()
    else:
        info = scenes.build(args.scene, r)
    over = {"max_depth": args.depth}
    if args.width:
        over["width"] = args.width
    if args.height:
        over["height"] = args.height
    if args.spp:
        over["spp"] = args.spp
    params = info.params(**over)
    r.set_tracer("interpreter" if args.jit == 0 else args.tracer)
    r.prepare()  # the kernel AUTO settles on, its background compile included (csg360: the lanes meanwhile)
    W, H, T = params.width, params.height, args.tile_rows
    band = wl.default_band(world) if args.band == "auto" else tuple(int(x) for x in args.band.split(":"))
    args.band_w = band if world > 1 else (0, 0)
    r.set_band_weight(*args.band_w)
    lr = wl.local_rows(H, T, world, args.band_w)
    # the same two-buffer / two-stream / event code runs on either backend, so a gloo
    # rehearsal on one GPU executes what the RCCL run on 8 GPUs does
    pipelined = world > 1 and not args.no_pipeline
    if args.frames_in_flight is None:
        args.frames_in_flight = 2 if pipelined else 1
    # two render buffers when pipelined: frame k+1 renders while frame k is gathered; with F frames
    # in flight, F buffers and F render streams
    nbuf = max(args.frames_in_flight, 2 if pipelined else 1)
    outs = [torch.empty((lr, W, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    seg = torch.zeros(1, dtype=torch.int64, device=dev)
    stacked = gathered = frame = None
    if world > 1 and rank == 0:
        # one rank-major buffer; the gather writes each rank's tiles into its slice
        stacked = torch.empty((world, lr, W, 4), dtype=torch.float32, device="cpu" if gloo else dev)
        gathered = list(stacked.unbind(0))
        frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    # render streams (one per buffer when frames overlap), then the gather + assemble
    # stream (RCCL's stream follows the current one).  N > 1: a created stream made
    # current, not the default stream: kernels on the default stream leave the two
    # render streams sharing a hardware queue (the box has 4), so frame k+1 no longer
    # overlaps frame k's tail (tools/root_step.py --streams null vs bench, N = 8:
    # csg32 share 0.437 vs 0.399 ms, csg256 chain 1.77 vs 1.66 ms)
    rss = [torch.cuda.Stream(dev) for _ in range(nbuf)] if args.frames_in_flight > 1 else None
    if world > 1:
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    cs = torch.cuda.current_stream(dev)
    if rss is None:
        rss = [torch.cuda.Stream(dev) if pipelined else cs] * nbuf
    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    rendered = [torch.cuda.Event() for _ in outs]
    released = [None for _ in outs]  # gather of the frame that last used the buffer
    frame_no = [0]

    def step(i=None):
        b = frame_no[0] % len(outs)
        frame_no[0] += 1
        out = outs[b]
        rs = rss[b]
        if released[b] is not None:
            rs.wait_event(released[b])
        if i is not None:
            k_start[i].record(rs)
        r.render_rows_device(params, out.data_ptr(), T, rank, world, rs.cuda_stream, seg.data_ptr())
        if i is not None:
            k_end[i].record(rs)
        if world > 1:
            if pipelined:
                rendered[b].record(rs)
                cs.wait_event(rendered[b])
            src = out.cpu() if gloo else out
            if rank == 0:
                dist.gather(src, gather_list=gathered, dst=0)
                g = stacked.to(dev, non_blocking=False) if gloo else stacked
                wl.assemble_rows_device(g.data_ptr(), frame.data_ptr(), W, H, T, world, cs.cuda_stream, args.band_w)
            else:
                dist.gather(src, dst=0)
            if pipelined:
                ev = torch.cuda.Event()
                ev.record(cs)
                released[b] = ev

    # Clock ramp: an idle GPU starts each run at low clocks and reaches its steady
    # clock over the first ~0.3 s of work (csg32 launches 3.84 -> 3.28 ms over the
    # first 8 frames in a rocprofv3 trace).  Untimed frames until that much wall
    # time has passed (at most 200), then the W warmup steps, then the K timed ones.
    # The count is fixed from the first frame's time and agreed over the ranks (every
    # rank must run the same number of steps: each holds a collective).
    prewarm = 0
    if args.prewarm_s > 0:
        step()  # the first frame may include loading the scene's code object: not timed
        torch.cuda.synchronize()
        t_pw = time.perf_counter()
        step()
        torch.cuda.synchronize()
        frame_s = max(time.perf_counter() - t_pw, 1e-4)
        n_pw = torch.tensor([min(200, int(args.prewarm_s / frame_s) + 1)], dtype=torch.int64,
                            device="cpu" if gloo else dev)
        if world > 1:
            dist.all_reduce(n_pw, op=dist.ReduceOp.MAX)
        prewarm = 2 + int(n_pw.item())
        for _ in range(prewarm - 2):
            step()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    seg.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    coll = "cpu" if gloo else dev  # gloo reduces host tensors
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=coll)
    segs_total = seg.clone().to(coll)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(segs_total, op=dist.ReduceOp.SUM)
    elapsed_s = float(elapsed.item())
    segs_local = int(seg.item())
    segs_all = int(segs_total.item())
    k_ms = sum(k_start[i].elapsed_time(k_end[i]) for i in range(args.steps)) / args.steps
    # executed work of this rank's share: one more frame with the counting variant of
    # the same kernel, outside the timed region (wo_renderer_count_work)
    work = None
    if rank == 0 and info.mode == wl.MODE_PATHTRACE and not args.no_count_work:
        work = r.count_work(params, T, rank, world)
        if work["segments"] * args.steps != segs_local:
            print(f"[bench] work counters traced {work['segments']} segments, the timed frames "
                  f"{segs_local / args.steps}", file=sys.stderr)

    verified = None
    if args.verify and rank == 0:
        import numpy as np
        full = r.render(params)
        got = (frame if world > 1 else outs[(frame_no[0] - 1) % len(outs)][:H]).cpu().numpy()
        verified = bool(np.array_equal(got, full))
        if not verified:
            bad = int((got != full).any(axis=-1).sum())
            print(f"[bench] VERIFY FAILED: {bad} pixels of the assembled frame differ from a full render",
                  file=sys.stderr)
    if world > 1:
        flag = torch.tensor([0 if verified is False else 1], dtype=torch.int32, device="cpu" if gloo else dev)
        dist.broadcast(flag, src=0)
        verified_all = bool(flag.item())
    else:
        verified_all = verified is not False

    if rank == 0:
        parallelism = (f"row-cyclic tiles x{world}" + (f" + {'gloo (host-staged)' if gloo else 'RCCL'} gather" if world > 1 else "")
                       + (" overlapped with the next frame's render" if pipelined else "")
                       + (f"; {world} ranks stacked on {ndev} GPU(s) (rehearsal)" if ranks_stacked else ""))
        line = report_line(args, r, info, params, world, elapsed_s, segs_all, segs_local, k_ms, work,
                           {"parallelism": parallelism, "ranks": world, "devices": min(world, ndev),
                            "launcher": "torchrun" if world_env else "none",
                            "frames_in_flight": args.frames_in_flight, "prewarm_frames": prewarm,
                            **({"row_bands": f"{args.band_w[0]}:{args.band_w[1]}",
                                "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")} if world > 1 else {})})
        if verified is not None:
            line["verified_vs_full_render"] = verified
        if world == 1 and info.mode == wl.MODE_PATHTRACE and not args.no_draw_frame:
            line["draw_frame"] = draw_frame_leg(r, params, args, line["fps"])
        if world == 1 and args.scene == "csg32" and args.side_scenes and not (args.width or args.height or args.spp):
            for name in [x for x in args.side_scenes.split(",") if x]:
                line[name.replace("csg32_", "")] = side_scene(name, args, dev)
        print(json.dumps(line), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()
    if not verified_all:
        sys.exit(3)


def draw_frame_leg(r, params, args, kernel_fps):
    """The product's frame rate: frames through wo_renderer_draw_frame (renderer.c:2085-2219's
    replacement), i.e. render + present encode + map-back to pinned host memory, each frame
    presented.  The pipeline is drained before and after the timed frames, so the time holds
    exactly `draw_frames` renders and the last frame's map-back.  Stamps of the same frames
    (HIP events of the pipeline) give the render and map-back times."""
    r.set_draw_params(params, pin_time=True)
    for _ in range(3):
        r.draw_frame()
    r.finish()
    n = max(args.draw_frames, 2)
    t0 = time.perf_counter()
    for _ in range(n):
        r.draw_frame()
    r.finish()
    dt = time.perf_counter() - t0
    r.set_frame_stamps(True)
    for _ in range(min(n, 20)):
        r.draw_frame()
    r.finish()
    st = r.frame_stamps()
    r.set_frame_stamps(False)
    fps = n / dt
    out = {"fps": round(fps, 3), "ms_per_frame": round(dt / n * 1e3, 4), "frames": n,
           "vs_kernel_fps": round(fps / kernel_fps, 4) if kernel_fps else None,
           "map_back": "present encode (B8G8R8A8 sRGB) + D2H to pinned host memory on a copy stream; "
                       "float frame on demand"}
    if len(st) > 2:
        import statistics
        out["stamps"] = {
            "frames": len(st),
            "render_ms_median": round(statistics.median(e - b for b, e, _ in st), 4),
            "map_back_ms_median": round(statistics.median(m - e for _, e, m in st), 4),
            "render_gap_ms_median": round(statistics.median(st[k + 1][0] - st[k][1] for k in range(len(st) - 1)), 4),
            "next_render_inside_map_back": sum(1 for k in range(len(st) - 1) if st[k + 1][0] < st[k][2]),
        }
    return out


def side_scene(name, args, dev):
    """Another BASELINE scene at the headline's size, timed like the headline (N = 1, same
    steps, HIP events on the launch stream) in the same invocation: ms_per_step, value and
    the executed-work roofline."""
    import torch

    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl
    r = wl.Renderer(f"side-{name}", max_nodes=4096)
    info = scenes.build(name, r)
    params = info.params(max_depth=args.depth)
    r.set_tracer("interpreter" if args.jit == 0 else args.tracer)
    r.prepare()
    W, H, T = params.width, params.height, args.tile_rows
    out = torch.empty((wl.local_rows(H, T, 1), W, 4), dtype=torch.float32, device=dev)
    seg = torch.zeros(1, dtype=torch.int64, device=dev)
    cs = torch.cuda.current_stream(dev)
    k0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            k0[i].record(cs)
        r.render_rows_device(params, out.data_ptr(), T, 0, 1, cs.cuda_stream, seg.data_ptr())
        if i is not None:
            k1[i].record(cs)

    step()
    torch.cuda.synchronize()
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    seg.zero_()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    segs = int(seg.item())
    k_ms = sum(k0[i].elapsed_time(k1[i]) for i in range(args.steps)) / args.steps
    work = None if args.no_count_work else r.count_work(params, T, 0, 1)
    sub_args = argparse.Namespace(**vars(args))
    sub_args.scene, sub_args.no_cpu_baseline = name, True
    line = report_line(sub_args, r, info, params, 1, elapsed, segs, segs, k_ms, work, {})
    r.close()
    return {k: line[k] for k in ("value", "unit", "ms_per_step", "fps", "segments_per_frame", "roofline")} | {
        "workload": line["config"]["workload"]}


def report_line(args, r, info, params, world, elapsed_s, segs_all, segs_local, k_ms, work, cfg_extra):
    """The JSON line (rank 0): value = segments of the whole frame over the max-over-ranks
    wall time; roofline of the dominant kernel from its per-launch time k_ms and the
    segments one launch traced (segs_local over the steps)."""
    from csgrenderer_amd import wololo as wl
    W, H, T = params.width, params.height, args.tile_rows
    band = getattr(args, "band_w", (0, 0))
    lr = min(wl.rank_bands(H, T, 0, world, band) * T, wl.local_rows(H, T, world, band))  # rank 0's rows
    steps = args.steps
    ms_per_step = elapsed_s / steps * 1e3
    samples = W * H * (params.spp if info.mode == wl.MODE_PATHTRACE else 1)
    if info.mode == wl.MODE_PATHTRACE:
        value = segs_all / elapsed_s / 1e6
        seg_launch = segs_local / steps
        brute_tf = seg_launch * info.flop_per_segment / (k_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": None, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": None,
                "traffic": None,
                "kernel": {"jit": "wo_jit_pathtrace", "lanes": "pathtrace_lanes_kernel"}.get(r.trace_path(),
                                                                                          "pathtrace_kernel"),
                "kernel_ms": round(k_ms, 4), "segments_per_launch": segs_local // steps,
                "trace_path": r.trace_path(),
                # the code object the timed launches ran (its key and resources), so a
                # profile or a traffic figure can be matched to it
                "kernel_object": r.kernel_info(),
                "brute_force_flop_per_segment": info.flop_per_segment,
                "brute_force_achieved": round(brute_tf, 3),
                "brute_force_frac": round(brute_tf / PEAK_FP32_TFLOPS, 4)}
        if work is not None:
            eval_ops = None
            if r.trace_path() == "jit":
                m = re.search(r"// wo_eval_ops_per_event (\d+)", r.jit_source() or "")
                eval_ops = int(m.group(1)) if m else None
            ex = executed_flop(work, info, r.trace_path(), eval_ops)
            ex_tf = ex / work["segments"] * seg_launch / (k_ms * 1e-3) / 1e12
            roof.update({"achieved": round(ex_tf, 3), "frac": round(ex_tf / PEAK_FP32_TFLOPS, 4),
                         "basis": "executed work (counted tests priced per SURVEY.md 8(d); a swept event "
                                  "priced at the emitted root evaluation's operations"
                                  + (f", {eval_ops} per event)" if eval_ops else ")"),
                         "executed_flop_per_segment": round(ex / work["segments"], 2),
                         "work_per_segment": {k: round(v / work["segments"], 4) for k, v in work.items()
                                              if k != "segments" and not k.startswith("cyc_")}})
        else:
            roof.update({"achieved": roof["brute_force_achieved"], "frac": roof["brute_force_frac"],
                         "basis": "brute force (every primitive on every segment, SURVEY.md 8(d))"})
    else:
        value = W * H * steps / elapsed_s / 1e6
        bytes_launch = lr * W * 16
        achieved = bytes_launch / (k_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": None, "kernel": "ubershader_kernel",
                "kernel_ms": round(k_ms, 5)}
    # the store stream (16 B/pixel) against HBM, for the record
    hbm_gbs = lr * W * 16 / (k_ms * 1e-3) / 1e9
    if args.pmc_json and os.path.exists(args.pmc_json):
        try:
            pmc = json.load(open(args.pmc_json))
            key = f"{args.scene}:{W}x{H}:{params.spp}:{world}:{roof.get('trace_path', 'ubershader')}"
            if key in pmc:
                ent = pmc[key]
                if isinstance(ent, dict):
                    # recorded with the profiled kernel's key: used only for the same code object
                    ko = roof.get("kernel_object") or {}
                    if ent.get("kernel_key") == ko.get("key"):
                        roof["traffic"] = ent["bytes"]
                        roof["traffic_kernel_key_match"] = True
                    else:
                        roof["traffic_kernel_key_match"] = False
                        roof["traffic_recorded_for"] = ent.get("kernel_key")
                else:
                    roof["traffic"] = ent  # a round-5 figure, recorded without a kernel key
        except Exception as e:  # report, don't fail the bench
            print(f"[bench] pmc json unreadable: {e}", file=sys.stderr)
    cpu = None
    if world == 1 and not args.no_cpu_baseline and info.mode == wl.MODE_PATHTRACE:
        cpu = cpu_baseline(r, params, args.cpu_seconds)
    shape = f" ({info.shape})" if info.shape else ""
    cfg = {"workload": f"{info.name}{shape}: {W}x{H}, {params.spp} spp, {params.max_depth} bounces, "
                       f"{info.spheres} spheres + {info.halfspaces} half-spaces, {info.binops} binops",
           "scene": info.name, "width": W, "height": H, "spp": params.spp,
           "max_depth": params.max_depth, "tile_rows": T}
    cfg.update(cfg_extra)
    cfg["hip_runtime"] = wl.load().wo_hip_runtime_version()
    return {
        "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": cfg,
        "fps": round(steps / elapsed_s, 3),
        "msamples_per_s": round(samples * steps / elapsed_s / 1e6, 3),
        "segments_per_frame": segs_all // steps,
        "roofline": roof,
        "roofline_hbm_store": {"bound": "hbm", "achieved": round(hbm_gbs, 3), "peak": PEAK_HBM_GBS,
                               "unit": "GB/s", "frac": round(hbm_gbs / PEAK_HBM_GBS, 6)},
        "cpu_baseline": cpu,
    }


def single_process(args):
    """N GPUs from one process through the C API: wo_renderer_set_devices(N) puts rank i
    on device i (its own stream and buffers; ranks stack when N exceeds the visible
    GPUs, with --stack-ranks), and a step is one wo_renderer_render_frame_device: every
    rank renders its row-cyclic tiles, ranks 1..N-1 copy their share into rank 0's
    gather buffer (peer DMA over xGMI), rank 0 assembles the frame in its HBM.
    Consecutive frames alternate two gather buffers, so frame k+1 renders while frame
    k is gathered.  The roofline's kernel time is the whole step here (the ranks'
    launches run on the library's streams)."""
    import numpy as np
    import torch

    from csgrenderer_amd import scenes
    from csgrenderer_amd import wololo as wl

    n = args.gpus
    ndev = visible_devices()
    if ndev < n and not args.stack_ranks:
        fail(f"--single-process --gpus {n} needs {n} GPUs, {ndev} visible (--stack-ranks to rehearse on fewer)")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    r = wl.Renderer("bench-sp", max_nodes=4096)
    info = scenes.sphere256() if args.scene == "sphere256" else scenes.build(args.scene, r)
    over = {"max_depth": args.depth}
    for k in ("width", "height", "spp"):
        if getattr(args, k):
            over[k] = getattr(args, k)
    params = info.params(**over)
    r.set_tracer("interpreter" if args.jit == 0 else args.tracer)
    if r.set_devices(n) != n or r.device_count() != n:
        fail(f"wo_renderer_set_devices({n}) failed: {wl.last_error()}")
    r.prepare()
    W, H = params.width, params.height
    frames = [torch.empty((H, W, 4), dtype=torch.float32, device=dev) for _ in range(2)]
    cs = torch.cuda.current_stream(dev)
    fno = [0]

    def step():
        r.render_frame_device(params, frames[fno[0] & 1].data_ptr(), cs.cuda_stream)
        fno[0] += 1

    step()  # the first frame may include loading the scene's code object
    torch.cuda.synchronize()
    t_pw = time.perf_counter()
    prewarm = 1
    while args.prewarm_s > 0 and prewarm < 200 and time.perf_counter() - t_pw < args.prewarm_s:  # clock ramp
        step()
        torch.cuda.synchronize()
        prewarm += 1
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    r.take_segments()  # the warm-up frames' count
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    elapsed_s = t1 - t0
    segs = r.take_segments()
    peers = sorted({r.peer_mode(i) for i in range(1, n)}) if n > 1 else []
    last = frames[(fno[0] - 1) & 1].cpu().numpy()
    r.set_devices(1)  # the counting frame and the verification render run on one rank
    work = None
    if info.mode == wl.MODE_PATHTRACE and not args.no_count_work:
        work = r.count_work(params, args.tile_rows, 0, 1)
    verified = None
    if args.verify:
        full = r.render(params)
        verified = bool(np.array_equal(last, full))
        if not verified:
            bad = int((last != full).any(axis=-1).sum())
            print(f"[bench] VERIFY FAILED: {bad} pixels of the assembled frame differ from a one-rank render",
                  file=sys.stderr)
    k_ms = elapsed_s / args.steps * 1e3
    args_rows = args.tile_rows
    args.tile_rows = 4  # the library's frames use 4-row tiles
    if n > 1:
        args.no_cpu_baseline = True  # the CPU baseline is an N = 1 figure
        args.pmc_json = None  # the committed PMC traffic is per N = 1 launch
    line = report_line(args, r, info, params, 1, elapsed_s, segs, segs, k_ms, work,
                       {"parallelism": f"row-cyclic tiles x{n}, one process, C API (wo_renderer_set_devices)"
                                       + (f", share gather by {'/'.join(peers)}" if peers else "")
                                       + (f"; {n} ranks stacked on {ndev} GPU(s) (rehearsal)" if ndev < n else ""),
                        "ranks": n, "devices": min(n, ndev), "launcher": "single-process",
                        "frames_in_flight": 2})
    args.tile_rows = args_rows
    line["n_gpus"] = n
    line["roofline"]["kernel_ms_basis"] = "whole step (all ranks' launches, gather and assembly)"
    if verified is not None:
        line["verified_vs_full_render"] = verified
    print(json.dumps(line), flush=True)
    r.close()
    if verified is False:
        sys.exit(3)


# SURVEY.md 8(d) prices: ray-sphere test 30 flop, ray-half-space 12, CSG combine 4 per
# binop (one root evaluation per swept event; the lane tracer's union count is one
# update), shading + scatter 40 per segment.  A BOUND test is the sphere test's
# centre-to-line part without the root: priced 20.  The specialised kernel states the
# operations its root evaluation runs per swept event (masked compares, a decision
# list or the union count's update: `eval_ops`, scene_jit.c), which replaces the
# 4-per-binop price where it is known.
def executed_flop(work, info, path, eval_ops=None):
    combine = 4 if path == "lanes" else (eval_ops if eval_ops else 4 * info.binops)
    return (30 * work["sphere_tests"] + 12 * work["halfspace_tests"] + 20 * work["bound_tests"]
            + combine * work["sweep_steps"] + 40 * work["segments"])


def cpu_baseline(r, params, budget_s: float):
    """The CPU oracle (oracle/oracle.c, a scalar C restatement of the same path) on a
    bounded sample of the same frame: whole rows from the middle of the image, as many
    as fit the time budget, on the host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    nthreads = pyoracle.nthreads_default()
    prog, nrec, _ = r.program()
    mats, nm = r.materials()
    fr = r.frame_desc(params)
    # whole rows starting at the middle of the frame, wrapping, until the budget is spent
    start = params.height // 2
    row = start
    rows = 0
    segs = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s and rows < params.height:
        n = min(nthreads // 4 + 1, params.height - row, params.height - rows)
        _, s = pyoracle.pathtrace_rows(prog, nrec, mats, nm, fr, row, n, nthreads=nthreads)
        segs += s
        rows += n
        row = (row + n) % params.height
    dt = time.perf_counter() - t0
    return {"value": round(segs / dt / 1e6, 4), "unit": "Mrays/s", "cores": nthreads, "kind": "port",
            "host_cpus": pyoracle.host_cpus(), "cpu_quota": pyoracle.cpu_quota(),
            "threads_from": pyoracle.threads_source(),
            "sample": f"{rows} of {params.height} rows (from row {start}, wrapping) of the "
                      f"same {params.width}x{params.height} frame, {params.spp} spp, {params.max_depth} bounces; "
                      f"{segs} segments in {dt:.1f} s"}


if __name__ == "__main__":
    main()
