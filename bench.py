"""Headline benchmark: YOLOv11n eval forward + on-device NMS, 640x640, batch 32 per GPU.

BASELINE.json metric: images/sec at 640x640 batch 32, v11_n, 1/2/4/8 MI355X.
A step = one pass of the hot path over one batch resident in HBM: the HIP
forward (yh_forward, replayed as a HIP graph), the on-device NMS (yh_nms) and,
for N > 1, the RCCL gather of the fixed-size detection buffers to rank 0.
By default steps are pipelined (yolo_hip.pipeline) over 3 forward lanes - three
engines (own workspace and HIP graphs, same weights), batch k on lane k % 3 -
plus one NMS stream: the forwards of consecutive batches overlap, so one
batch's latency-bound 40x40 / 20x20 layers share the chip with another's
large layers, and the NMS (+ gather) of batch k runs beside them. Every batch
still gets its full forward and NMS inside the timed region. --lanes 1 is the
two-stream pipeline (forward k+1 beside NMS k); --serial runs forward and NMS
back to back on one stream.
Data-parallel: every rank processes its own batch of 32 (weak scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Prints ONE JSON line on rank 0 (fields per the driver contract), including
`roofline` (dominant kernel family: the dense 3x3 implicit-GEMM convs, timed
with HIP events per launch on the forward's stream) and `cpu_baseline` (the CPU
oracle, fp32 forward + NMS, on the host cores, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "yolo-infer-pt_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}  # dense, spec
DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(variant):
    from nets import nn
    from yolo_hip import synth
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{variant}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    return model.eval()


def roofline(eng, args, batch, prof_steps, x, y):
    """Per-launch HIP-event timing of every op over `prof_steps` forwards (same stream)."""
    eng.profile(True)
    eng.profile_reset()
    for _ in range(prof_steps):
        eng.forward(x, out=y)
    eng.profile(False)
    ops = eng.units(batch, args.size, args.size)   # launch units (one op each)
    by_cls = {}
    for o in ops:
        c = by_cls.setdefault(o["cls"], dict(ms=0.0, bytes=0.0, flops=0.0, launches=0, attain_ms=0.0))
        avg_ms = o["ms"] / max(1, o["calls"])
        c["ms"] += avg_ms
        c["bytes"] += o["bytes"]
        c["flops"] += o["flops"]
        c["launches"] += 1
        # every class is scored against the roof of the arithmetic it runs: the 16-bit handles'
        # kernels (convs and every fused kernel) run bf16/fp16 MFMA, the fp32 handle fp32/fp64
        peak_tf = MFMA_PEAK_TFLOPS[args.dtype]
        c["attain_ms"] += max(o["bytes"] / (HBM_PEAK_GBS * 1e9), o["flops"] / (peak_tf * 1e12)) * 1e3
    total = sum(c["ms"] for c in by_cls.values())
    total_bytes = sum(c["bytes"] for c in by_cls.values())
    total_flops = sum(c["flops"] for c in by_cls.values())
    total_attain = sum(c["attain_ms"] for c in by_cls.values())
    for k, c in sorted(by_cls.items(), key=lambda kv: -kv[1]["ms"]):
        log(f"  {k:10s} {c['launches']:3d} launches  {c['ms'] * 1e3:8.1f} us/fwd ({100 * c['ms'] / total:4.1f}%)  "
            f"{c['bytes'] / c['ms'] / 1e6:7.0f} GB/s  {c['flops'] / c['ms'] / 1e9:7.1f} TFLOP/s  "
            f"attainable {100 * c['attain_ms'] / c['ms']:4.1f}%")
    dom = by_cls["conv3x3"]
    # the family's binding roof: HBM below the ridge (v11_n/s at 640), MFMA above (v11_x at 1280)
    peak_tf = MFMA_PEAK_TFLOPS[args.dtype]
    mfma_bound = dom["flops"] / (peak_tf * 1e12) > dom["bytes"] / (HBM_PEAK_GBS * 1e9)
    if mfma_bound:
        achieved, peak, unit, bound = dom["flops"] / dom["ms"] / 1e9, peak_tf, "TFLOP/s", "mfma"
    else:
        achieved, peak, unit, bound = dom["bytes"] / dom["ms"] / 1e6, HBM_PEAK_GBS, "GB/s", "hbm"
    traffic, traffic_src = pmc_traffic("conv3x3", args)
    return dict(bound=bound, achieved=round(achieved, 1), peak=peak, unit=unit,
                frac=round(achieved / peak, 4), traffic=traffic, traffic_source=traffic_src,
                algorithmic_flops_per_launch=round(dom["flops"] / dom["launches"]),
                kernel=("dense 3x3 convs: conv_mx (staged weights) / conv_mxr (resident weights) implicit GEMM "
                        "on v_mfma_f32_32x32x16, LDS-DMA patch staging, plan autotuned per layer")
                if args.dtype != "fp32" else "dense 3x3 convs: conv_gemm (fp32 FMA implicit GEMM)",
                timing="HIP events around each launch on the forward's stream, eager (one forward at a time); "
                       f"{TRACE_PROFILE} holds the rocprofv3 per-dispatch trace of the same "
                       "forwards replayed as graphs (tools/fwd_trace.py + tools/trace_ops.py)",
                launches_per_step=dom["launches"],
                avg_launch_us=round(dom["ms"] * 1e3 / dom["launches"], 2),
                algorithmic_bytes_per_launch=round(dom["bytes"] / dom["launches"]),
                attainable_frac=round(dom["attain_ms"] / dom["ms"], 4),
                forward_kernel_ms=round(total, 4),
                # the whole forward against HBM: algorithmic bytes of every op per forward over the
                # summed kernel time (HIP events, one forward at a time) and 8 TB/s
                forward=dict(algorithmic_bytes=round(total_bytes), algorithmic_flops=round(total_flops),
                             kernel_ms=round(total, 4),
                             achieved_GBs=round(total_bytes / total / 1e6, 1),
                             frac_hbm=round(total_bytes / total / 1e6 / HBM_PEAK_GBS, 4),
                             attainable_frac=round(total_attain / total, 4),
                             launches=sum(c["launches"] for c in by_cls.values())),
                per_class={k: dict(launches=c["launches"], us=round(c["ms"] * 1e3, 1),
                                   algorithmic_MB=round(c["bytes"] / 1e6, 2),
                                   attainable_frac=round(c["attain_ms"] / c["ms"], 4))
                           for k, c in by_cls.items()})


PMC_ROUND = "r06"   # this round's committed PMC summaries (copies of the tools/pmc_*.sh outputs) come first
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_traffic_latest.json")
TRACE_PROFILE = "profiles/r06_fwd_trace_ops.txt"   # rocprofv3 per-dispatch trace of this round's library


def pmc_traffic(cls, args):
    """HBM bytes per launch of kernel family `cls` from the committed rocprofv3 PMC summary
    (FETCH_SIZE / WRITE_SIZE passes over tools/pmc_run.py, corrected per the gfx950 guide by
    tools/pmc_traffic.py); bench.py cannot collect PMC counters from inside its own process.
    profiles/<round>_pmc_traffic.json / pmc_traffic_latest.json (the headline configuration) or,
    for the other configs, profiles/[<round>_]pmc_traffic_<variant>_<size>_b<batch>_<dtype>.json
    (tools/pmc_config.sh). None unless a summary was collected on this bench's configuration."""
    want = (args.variant, args.size, args.batch, args.dtype)
    cfg_name = "pmc_traffic_%s_%d_b%d_%s.json" % want
    prof = os.path.join(ROOT, "profiles")
    for path in (os.path.join(prof, PMC_ROUND + "_pmc_traffic.json"), PMC_SUMMARY,
                 os.path.join(prof, PMC_ROUND + "_" + cfg_name), os.path.join(prof, cfg_name)):
        try:
            with open(path) as f:
                rec = json.load(f)
            cfg = rec.get("config", {"variant": "n", "size": 640, "batch": 32, "dtype": "bf16"})
            if (cfg["variant"], cfg["size"], cfg["batch"], cfg["dtype"]) != want:
                continue
            fam = rec["family"][cls]
            return round(fam["traffic_per_launch"]), (f"{os.path.relpath(path, ROOT)}: {rec['source']}; "
                                                      f"{rec['corrections']}; {fam['traffic_over_alg']:.2f}x algorithmic")
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def cpu_baseline(args, runs=3):
    """the build's CPU restatement of the forward (oracle/, fp32 functional
    forward with BN folded, torch.inference_mode()) plus the library's C++ host NMS (yh_nms_host,
    the contract torchvision's C++ kernel fills in the reference) on one batch of the bench's size,
    every host core this process may use, one warm-up then the median of `runs` timed runs. The
    forward and the NMS are timed separately and reported both apart and together."""
    import statistics
    from oracle.forward import Oracle
    from yolo_hip.engine import nms_host
    from yolo_hip.variants import VARIANTS

    # cores this process may use: the box's CPU share (OMP_NUM_THREADS is set to it there;
    # os.cpu_count() reports the whole machine), else the affinity mask
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS") or avail)
    threads = max(1, min(threads, avail))
    torch.set_num_threads(threads)
    model = build_model(args.variant)
    v = VARIANTS[args.variant]
    orc = Oracle(model.state_dict(), v.width, v.depth, v.csp, 80, dtype=torch.float32)
    B = args.batch
    g = torch.Generator().manual_seed(0)
    x = torch.rand(B, 3, args.size, args.size, generator=g)   # BASELINE.md section 3 inputs

    def once():
        t0 = time.perf_counter()
        with torch.inference_mode():
            y = orc(x)
        t1 = time.perf_counter()
        nms_host(y, threads=threads)
        return t1 - t0, time.perf_counter() - t1

    once()   # warm-up
    res = [once() for _ in range(runs)]
    fwd = statistics.median(r[0] for r in res)
    nms_s = statistics.median(r[1] for r in res)
    tot = statistics.median(r[0] + r[1] for r in res)
    return dict(value=round(B / tot, 3), unit="images/s", cores=threads, kind="port",
                cpu_model=_cpu_model(), host_cpus_visible=os.cpu_count(),
                forward_images_per_s=round(B / fwd, 3), forward_s=round(fwd, 3),
                nms_s=round(nms_s, 4), runs_s=[round(r[0] + r[1], 3) for r in res],
                sample=f"batch {B} (torch.rand seed 0, {args.size}x{args.size}), v11_{args.variant} fp32 oracle "
                       f"forward (BN folded) + C++ host NMS (yh_nms_host); 1 warm-up + median of {runs} runs, "
                       f"{threads} threads, torch.inference_mode()")


def visible_gpus_without_hip():
    """GPUs this process could use, counted without initialising HIP (the self-launch parent must
    not: the ranks it spawns then start from a clean driver state). KFD topology nodes with SIMDs
    are the GPUs; HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES narrow them.
    None when the topology is not readable (each rank then checks its own ordinal)."""
    import glob
    n = 0
    try:
        for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            with open(f) as fh:
                props = dict(line.split()[:2] for line in fh if len(line.split()) >= 2)
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except (OSError, ValueError):
        return None
    if n == 0:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) started without a launcher: run N ranks, one per GPU, under
    torch.distributed.run as child processes and return its exit code. The reference's own
    multi-process entry is env-driven under a launcher (main.py:338-344, main.sh:1-2); here the
    bench provides the launcher itself. This parent makes no GPU call (it counts the GPUs from the
    KFD topology, visible_gpus_without_hip), so the ranks start from a clean process."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    log(f"bench: launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 50 steps: with 3 lanes the pipeline's fill and drain are a few % of a 20-step run
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variant", default="n")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU per step")
    ap.add_argument("--dtype", default="bf16", choices=sorted(DTYPES))
    ap.add_argument("--profile-steps", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--lanes", type=int, default=3,
                    help="forward lanes: engines whose forwards of consecutive batches overlap "
                         "(measured r01, v11_n b32: 1 -> 20.3k, 2 -> 23.2k, 3 -> 27.2k, 4 -> 25.2k img/s)")
    ap.add_argument("--nms-on-lane", action="store_true",
                    help="run each batch's NMS on its forward lane's stream (no separate NMS stream)")
    ap.add_argument("--input-ring", type=int, default=4,
                    help="distinct input batches the timed steps cycle through (> 256 MB of MALL in total)")
    ap.add_argument("--serial", action="store_true",
                    help="run forward and NMS back to back on one stream (no batch-to-batch overlap)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no HIP: gloo on the CPU and a stub step (the gather of empty detection buffers); "
                         "checks the launcher, rank layout, timing and JSON line without a GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        ngpu = None if args.dry_run else visible_gpus_without_hip()
        if ngpu is not None and ngpu < args.gpus:
            raise SystemExit(f"bench.py --gpus {args.gpus}: only {ngpu} GPU(s) visible")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torch.distributed.run (RANK + MASTER_ADDR set): a process group even at
    # world size 1, so the RCCL gather of the results runs on the device in every such run
    dist = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)
    if "WORLD_SIZE" in os.environ and args.gpus != world:
        log(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s); n_gpus = {world}")
    if args.dry_run:
        return dry_run(args, rank, world, dist)
    if local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) visible")
    if dist:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        # the barriers around the timed steps on a CPU (gloo) group: an RCCL barrier launches a
        # kernel, and a foreign kernel right before the timed steps slows the following milliseconds
        # of ours (profiles/r06_bench_marker_ab.txt); the results' gather stays on RCCL
        bar_group = torch.distributed.new_group(backend="gloo")
    dev = torch.device("cuda", local)
    dtype = DTYPES[args.dtype]

    from yolo_hip import synth
    from yolo_hip.dist import Gather
    from yolo_hip.engine import Engine, nms
    from yolo_hip.pipeline import DetectPipeline

    if args.serial:
        args.lanes = 1
    model = build_model(args.variant)
    B, S = args.batch, args.size
    engs = []
    for _ in range(args.lanes):
        e = Engine(*model._yh_arch, dev, dtype)
        e.load_module(model)
        e.reserve(B, S, S)
        engs.append(e)
    eng = engs[0]
    # synthetic scenes resident in HBM before timing: a ring of distinct batches per rank whose
    # total (4 x 78.6 MB at v11_n b32 640^2 bf16) exceeds the 256 MB MALL, so a step's input is
    # not left in the last-level cache by an earlier step
    ring = max(1, args.input_ring)
    xs = [synth.synth_scenes(B, S, S, seed=100 + rank + 1000 * k).to(dev, dtype) for k in range(ring)]
    x = xs[0]
    A = eng.num_anchors(S, S)
    y = torch.empty((B, 84, A), dtype=dtype, device=dev)
    gather = Gather(B, 300, dev, rank, world, slots=2 * args.lanes + 2)   # >= batches in flight

    post = (lambda d, c: gather(d, c)) if dist else None  # RCCL gather of the fixed-size results to rank 0
    for e in engs:   # tune + capture each lane's graphs one at a time, before any overlap
        e.forward(x, out=y)
        torch.cuda.synchronize()
    # result ring: each in-flight batch's dets / counts live in a slot allocated once (a batch's
    # results stay valid until the caller submits 2 x lanes more batches), no per-step allocation
    pipe = DetectPipeline(engs, B, S, S, post=post, nms_on_lane=args.nms_on_lane, result_ring=True)

    it = [0]

    def step():
        xk = xs[it[0] % ring]
        it[0] += 1
        if args.serial:
            eng.forward(xk, out=y)
            dets, counts = nms(y)
            extra = post(dets, counts) if dist else None
            return dets, counts, extra
        # forward of this batch overlaps the NMS (+ gather) of the previous one
        return pipe.submit(xk)[:3]

    # No marker kernel before the timed region: a torch fill kernel between the warm-up and the
    # timed steps (on the null stream or the NMS stream alike) cost the 20-step region ~6 %, and
    # 2-4 % even before the warm-up (profiles/r06_bench_marker_ab.txt). tools/trace_stats.py finds
    # the region in a trace as the dispatches between the idle gap of the synchronize and the end
    # marker below.
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier(group=bar_group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    t_sub = time.perf_counter() - t0   # host time of the submit loop (diagnostic, stderr)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier(group=bar_group)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    torch.zeros(1, device=dev).fill_(8.0)   # end marker (outside the timed region)
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    log(f"bench: timed region {elapsed * 1e3:.3f} ms, host submit loop {t_sub * 1e3:.3f} ms")
    dets, counts, extra = last
    kept = counts.cpu().tolist()
    gather_check = None
    if dist and rank == 0:
        # the last step's gathered rows of rank 0 are its own NMS results
        from yolo_hip.dist import pack
        gather_check = bool(torch.equal(extra[0], pack(dets, counts)))

    roof = None
    if not args.no_roofline:
        if rank == 0:
            log(f"per-class kernel time (HIP events, {args.profile_steps or args.steps} forwards, batch {B}):")
        roof = roofline(eng, args, B, args.profile_steps or args.steps, x, y)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        imgs = B * world * args.steps
        value = imgs / elapsed
        rec = {
            "metric": f"images/sec at {S}x{S} batch{B}, v11_{args.variant} (forward + on-device NMS)",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": f"synthetic (seeded scenes, a ring of {ring} distinct batches; calibrated synthetic weights)",
            "config": {"workload": f"yolo_v11_{args.variant} eval forward + NMS, {S}x{S}, {B} images per GPU per step",
                       "per_gpu_batch": B, "global_batch": B * world, "image_size": S,
                       "parallelism": f"dp{world}", "nms": "on-device, conf 0.001, iou 0.65, max_det 300"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "schedule": "serial" if args.serial else (
                "2-stream pipeline (forward k+1 overlaps NMS k)" if args.lanes == 1 else
                f"{args.lanes} forward lanes (forwards of consecutive batches overlap) + NMS stream"),
            "kept_last_step": kept[:4],
            "gather": (f"RCCL gather of packed detections to rank 0 over {world} rank(s), "
                       f"last step rank-0 rows match: {gather_check}") if dist else None,
        }
        print(json.dumps(rec), flush=True)
    if dist:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def dry_run(args, rank, world, dist):
    """The multi-rank skeleton of main() without HIP: gloo process group, a stub step that gathers
    an empty (B, 300, 6) detection buffer to rank 0, the same barrier / max-over-ranks timing and
    one JSON line on rank 0 (tests/test_bench_launch.py runs it at N = 2 on the CPU)."""
    from yolo_hip.dist import Gather
    if dist:
        torch.distributed.init_process_group("gloo")
    B = args.batch
    gather = Gather(B, 300, "cpu", rank, world, slots=2)
    dets = torch.zeros((B, 300, 6))
    counts = torch.full((B,), rank, dtype=torch.int32)
    for _ in range(args.warmup):
        gather(dets, counts)
    if dist:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = gather(dets, counts)
    if dist:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    if rank == 0:
        ranks_seen = [int(p[0, -1].item()) for p in got]
        print(json.dumps({"metric": "dry run (no HIP)", "value": round(B * world * args.steps / elapsed, 2),
                          "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dry_run": True, "ranks_gathered": ranks_seen,
                          "config": {"per_gpu_batch": B, "global_batch": B * world,
                                     "parallelism": f"dp{world}"}}), flush=True)
    if dist:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
