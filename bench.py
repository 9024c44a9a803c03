"""Headline bench: Mrays/s on the BASELINE.json synthetic K-triangle scene at 1920x1080
(primary + shadow rays), the roofline fraction of the dominant kernel against the memory
level that serves its bytes, and the reference's own multithreaded CPU path timed on this
host beside it.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one full 1920x1080 frame (one sample pass) traced and shaded, inputs (scene, BVH)
resident in HBM.  With N ranks every frame is partitioned (multigpu.py): rank r renders the
8-row bands dealt round-robin (rotated one slot per round) into its own HBM -- no collective on the data path (the
barriers around the timed region and the max-over-ranks of the elapsed time are the only
collectives).  The steps rotate over 16 scene replicas, each on its own stream ("frames in
flight"), so a frame's kernels overlap the next frames' -- a part of 1/N of one frame alone
is too small a grid to keep a GPU busy; `config.serial` times the same steps
on one stream, one frame after the other.  `value` = rays of the frames x steps /
max-over-ranks time.
The host framebuffer gather (every rank rendering its rows straight into one page-locked
shared frame) is timed separately ("gather"); the one-process host-buffer path of the CLI ("host_frame")
too -- neither is `value` (the PCIe-inclusive rates).
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

# Frames in flight: every step renders one frame, and the steps rotate over FRAMES_IN_FLIGHT
# scene replicas, each on its own stream, so one frame's kernels overlap the next frames' (a
# part of 1/N of a frame is too small a grid to fill the GPU on its own: DESIGN.md §6).  Each
# stream needs its own hardware queue (HIP's default is 4 per process, and streams beyond the
# queues share them and serialise: part (0, 8) 0.14 ms with 4 queues, 0.070 with 9;
# profiles/r03o_parts_queues.txt); raised to 17 -- the replicas' 16 streams + torch's own --
# before the HIP runtime starts.  Round 4: 16 frames in flight instead of 8 (a part of 1/8 of the
# frame 0.0522 -> 0.0501 ms, the full frame unchanged: profiles/r04f_parts_ab.jsonl).
FRAMES_IN_FLIGHT = 16
HW_QUEUES = int(os.environ.get("RTG_BENCH_HW_QUEUES", str(FRAMES_IN_FLIGHT + 1)))
if "--help" not in sys.argv and "-h" not in sys.argv:
    # (RTG_BENCH_QUEUES_AS_GIVEN=1: keep the environment's value, for the A/B)
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < HW_QUEUES and not os.environ.get("RTG_BENCH_QUEUES_AS_GIVEN"):
        os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "advanced-cpu-raytracing_amd")
sys.path.insert(0, PKG)

METRIC = "Mrays/sec + achieved HBM GB/s fraction, 1920×1080 primary+shadow rays"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, "HBM")
L2_PEAK_GBS = 34500.0      # MI355X L2 aggregate over the 8 XCDs (MI355X_MICROARCH.md, "L2 (per XCD)")
SWEEP_K = (1000, 10082, 100352, 1002528)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--K", type=int, default=100352, help="triangles in the synthetic height field")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--no-sweep", action="store_true", help="skip the K sweep (rank 0, N=1 only)")
    p.add_argument("--no-extras", action="store_true", help="skip gather / host-frame timings")
    p.add_argument("--config", default="headline", choices=["headline", "c2", "c3", "c3ton", "c4", "c5"],
                   help="BASELINE.json configuration (c2-c5: one frame = all camera samples)")
    p.add_argument("--inflight", type=int, default=0,
                   help="frames in flight (scene replicas / streams the steps rotate over); 0 = 16, "
                        "1 for c5")
    return p.parse_args()


CONFIG_DESC = {
    "c2": "C2 conductor Cornell box + OriginalPhong BRDF, 800x800, 1 spp, depth 6",
    "c3": "C3 70k-triangle mesh + area light, OriginalBlinnPhong, 1920x1080, 4 spp",
    "c3ton": "C3 on the reference's ton_Roosendaal scene (62k-triangle PLY + 2 meshes) + area light, "
             "OriginalBlinnPhong, 1920x1080, 4 spp",
    "c4": "C4 10k-triangle tree x 100 MeshInstances (~1M effective) + spherical env light, "
          "TorranceSparrow kdfresnel, 1920x1080, 16 spp",
    "c5": "C5 870k-triangle dielectric mesh + mirror sphere + Perlin ground, depth 5, 3840x2160, 64 spp",
}


def make_workload(args, out_dir, K=None):
    import scenes
    if args.config == "headline" or K is not None:
        K = K or args.K
        xml = scenes.synthetic_heightfield(out_dir, K=K, width=args.width, height=args.height)
        desc = (f"synthetic height field K={K} tris, {args.width}x{args.height}, 1 spp, 1 point light, "
                "default Blinn-Phong, primary+shadow rays")
        return xml, desc
    if args.config == "c2":
        xml = scenes.config_c2(out_dir, os.path.join(ROOT, "tests", "golden", "scenes", "cornell_conductors.xml"))
    elif args.config == "c3ton":
        xml = scenes.config_c3_ton(out_dir, os.path.join(ROOT, "tests", "golden", "scenes", "ton_Roosendaal_smooth_ply"))
    else:
        xml = getattr(scenes, "config_" + args.config)(out_dir)
    return xml, CONFIG_DESC[args.config]


def log(msg):
    """Progress on stderr (long configurations: keeps the run visibly alive)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- CPU baseline
def box_threads():
    """The host cores this process may use: the affinity mask, capped by OMP_NUM_THREADS
    (the GPU box sets it to the box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _median(v):
    v = sorted(v)
    return v[len(v) // 2]


# The CPU leg's sample per configuration: the whole frame, or a band of rows where the whole
# frame would take minutes (C5: 2.2 G rays; C4: 59 M rays through the restatement) -- about
# 10-30 s of CPU work per run.  C4 takes the restatement ("port"): the reference itself is
# undefined behaviour on MeshInstance scenes (instancedMesh.hpp:23 + raytracer.cpp:590) and
# crashes on C4.
CPU_SAMPLE = {"c4": {"rows": (404, 676), "reps": 2, "kind": "port"},
              "c5": {"rows": (1048, 1112), "reps": 1}}


def cpu_baseline(xml_dir, xml, count_rays, reps, rows=None, kind=None):
    """The reference's CPU path (oracle/_ref/refdriver: its own sources, row-band threads
    exactly as main.cpp:38-39,164-185 and each pixel's spp loop as renderThreadMain,
    main.cpp:42-121) on this host, in SURVEY §8d's two modes: A = the reference's THREAD_COUNT
    (8), B = every core of this box's share.  Per mode: the render alone (thread spawn -> join)
    and the reference-equivalent span main.cpp:138->199 (Raytracer copy + render + PNG encode).
    `rows`: a band of the frame (the rows each mode's threads cover exactly as main.cpp deals
    them); `count_rays(r0, r1)` gives the rays of those rows from the GPU's counting render.
    The CPU restatement ("port") when the reference build is absent or `kind` asks for it."""
    drv = os.path.join(ROOT, "oracle", "_ref", "refdriver")
    modes = {}
    kind = kind or ("reference" if os.path.exists(drv) else "port")
    for label, threads in (("A", 8), ("B", box_threads())):
        if kind == "reference":
            cmd = [drv, "bench", os.path.basename(xml), str(threads), str(reps), "0",
                   os.path.join(xml_dir, "refdriver_bench.png")]
            if rows:
                cmd += [str(rows[0]), str(rows[1])]
            out = subprocess.run(cmd, cwd=xml_dir, capture_output=True, text=True, timeout=900, check=True).stdout
            rec = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
            render_s, span_s = _median(rec["seconds"]), _median(rec["span_seconds"])
            r0, r1 = rec["rows"]
        else:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_bind as ob
            import rtgpu
            hs = rtgpu.HostScene(xml)
            h = hs.camera(0)["height"]
            r0, r1 = rows or (0, h)
            r1 = r0 + (r1 - r0) // threads * threads       # the rows main.cpp's threads would cover
            secs = []
            for _ in range(reps):
                t0 = time.perf_counter()
                ob.render(hs, rows=(r0, r1), threads=threads)
                secs.append(time.perf_counter() - t0)
            render_s = span_s = _median(secs)
            hs.close()
        rays = count_rays(r0, r1)
        modes[label] = {"threads": threads, "rows": [r0, r1], "rays": int(rays), "render_s": round(render_s, 4),
                        "span_s": round(span_s, 4), "mrays_s": round(rays / render_s / 1e6, 3),
                        "span_mrays_s": round(rays / span_s / 1e6, 3)}
        log(f"cpu baseline mode {label}: {threads} threads, rows {r0}-{r1}, {modes[label]['mrays_s']} Mrays/s")
    a = modes["A"]
    what = "the reference itself (oracle/_ref/refdriver)" if kind == "reference" else \
        "the CPU restatement (oracle/cpu_oracle.cpp, liboracle.so)"
    band = (f"rows {a['rows'][0]}-{a['rows'][1]} of the frame" if rows else "full frame")
    return {"value": a["mrays_s"], "unit": "Mrays/s", "cores": a["threads"], "kind": kind,
            "sample": f"{band} of {os.path.basename(xml)} ({a['rays']} rays, every sample per pixel) x {reps} reps "
                      f"per mode, {what}; value = mode A (THREAD_COUNT=8, render only: spawn->join, "
                      f"main.cpp:164-185); mode B = the box's {modes['B']['threads']} cores; span = "
                      f"main.cpp:138->199 (Raytracer copy + render + PNG)",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(), "modes": modes}


# ----------------------------------------------------------------------------- timing
def measure(render, torch, steps, warmup, barrier, serial=None):
    """Wall time of exactly `steps` frames between barrier + synchronize on both sides (no
    event records inside the timed loop: they cost ~0.01 ms per frame, tools/diag_streams.py);
    `render(k)` issues step k (with frames in flight, on the stream of replica k % F -- the
    device-wide synchronize waits for all of them).  From a separate untimed pass of
    `serial()` (one replica, one stream) with an event pair around each frame: the mean GPU
    time of one frame alone."""
    import inspect
    if len(inspect.signature(render).parameters) == 0:
        r0 = render
        render = lambda k: r0()  # noqa: E731
    serial = serial or (lambda: render(0))
    for k in range(warmup):
        render(k)
        torch.cuda.synchronize()
        log(f"warmup {k + 1}/{warmup}")
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = t0
    for k in range(steps):
        render(k)
        if k % 8 == 7 and time.perf_counter() - last > 20.0:    # long steps (C5): keep the run visibly alive
            last = time.perf_counter()
            log(f"step {k + 1}/{steps}")
    measure.issue_s = time.perf_counter() - t0    # host time to issue the steps (launch-bound if ~elapsed)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    stream = torch.cuda.current_stream()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    for k in range(steps):
        starts[k].record(stream)
        serial()
        ends[k].record(stream)
    torch.cuda.synchronize()
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / steps
    return elapsed, kern_ms


def kernel_times(ds, torch, render_timed, steps):
    """Per-kernel durations: HIP events recorded by the library around each kernel on the
    render's stream (RTG_RENDER_TIMING), averaged over `steps` frames."""
    acc = {}
    for _ in range(steps):
        render_timed()
        for k, v in ds.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    return {k: v / steps for k, v in acc.items()}


def kernel_bytes(st, W, H):
    """Algorithmic bytes per launch of each kernel (32 B per node visit,
    36 B per triangle test, 64 B per ray = ray in + hit out, 15 B per pixel written; the
    shadow rays' 4-wide BVH nodes are 128 B: four child boxes + references, RTG_SHADOW_MODE 3, the
    default build).  k_frame (the fused layout's one kernel per sample pass, the headline's
    default since round 5): camera + shadow rays + pixels."""
    ext_rays = st["camera_rays"] + st["secondary_rays"]
    ext = 32 * st["node_visits"] + 36 * st["tri_tests"] + 64 * ext_rays
    shd = (32 * st["shadow_node_visits"] + 128 * st.get("shadow_wide_visits", 0) + 36 * st["shadow_tri_tests"]
           + 64 * st["shadow_rays"])
    return {"k_primary": ext, "k_shadow": shd, "k_shade_shadow": shd + 15 * W * H, "k_render": ext + shd + 15 * W * H,
            "k_frame": ext + shd + 15 * W * H, "tree_levels": ext + shd, "frame": ext + shd + 15 * W * H}


def pmc_summary(kernel, K, world, share=1.0, workload="headline"):
    """Counter-measured bytes per launch of `kernel` for the K-triangle headline scene (or the
    BASELINE configuration `workload`) from the newest committed summary (profiles/r*_pmc*.json,
    tools/pmc_kernels.py over separate rocprofv3 --pmc passes of this bench): HBM traffic =
    2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction, MI355X_MICROARCH.md), L2 hit rate from
    TCC_HIT / TCC_MISS, L2 requests, vL1D hit rate, SQ instruction counts and wave-cycle split.
    A timed stage that spans several kernels (deferred leaves, the ray-tree levels) takes the
    summary's per-pass stage sums ("stage:<name>").  None if absent.

    N > 1 (no committed profile of a 1/N part): the N = 1 counters with every extensive count
    (instructions, bytes, requests, waves) scaled by this rank's share of the frame's rays and
    the ratios (hit rates, wave-cycle fractions) kept -- labelled as such in `source`."""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc*.json"))):
        rec = json.load(open(f))
        cfg = rec.get("config", {"K": 100352, "n_gpus": 1})
        if cfg.get("workload", "headline") != workload or cfg.get("n_gpus", 1) != world:
            continue
        if workload == "headline" and cfg.get("K") != K:
            continue
        # the timed kernels (the counting pass runs the <true> = STATS instantiations)
        v = (rec["kernels"].get("stage:" + kernel) or rec["kernels"].get(kernel + "<false>") or
             rec["kernels"].get(kernel))
        if v is None:     # a kernel whose first template argument is not STATS (C2's k_render<FEAT>)
            named = [n for n in rec["kernels"] if n.startswith(kernel + "<") and n != kernel + "<true>"]
            v = rec["kernels"][named[0]] if len(named) == 1 else None
        if v and "traffic_bytes" in v:
            best = dict(v, source=os.path.basename(f))
            best.setdefault("l2_request_bytes", 128 * v["l2_requests"] if "l2_requests" in v else None)
            if best["l2_request_bytes"] is None:
                del best["l2_request_bytes"]
    if best is None and world > 1:
        one = pmc_summary(kernel, K, 1, workload=workload)
        if one:
            best = {k: (v * share if isinstance(v, (int, float)) and not k.endswith(("_frac", "_rate")) else v)
                    for k, v in one.items()}
            best["source"] = (f"{one['source']} (N=1 counters; extensive counts x {share:.4f}, this rank's share "
                              f"of the frame's rays)")
    return best


CLOCK_GHZ = 2.4            # MI355X engine clock (MI355X_MICROARCH.md)
SIMDS, CUS = 1024, 256     # 256 CUs x 4 SIMDs
VALU_CYC = 2.0             # one wave64 VALU instruction per 2 cycles per SIMD ("v_fma_f32 (wave64)")


def limiter(pmc, kernel_ms):
    """Which unit limits the kernel, from its counters (profiles/r*_pmc_K*.json, one rocprofv3
    --pmc pass per counter group) and its live duration: the busy fraction of each unit
    = work / (units x cycles of the launch).  VALU: SQ_INSTS_VALU x 2 cycles over the 1024
    SIMDs; SALU: SQ_INSTS_SALU over the 256 CUs' scalar units; L2: TCC_REQ x 128 B against the
    34.5 TB/s aggregate; HBM: the corrected FETCH + WRITE bytes against 8 TB/s.  A unit at 70 %
    or more is the bound; when none is and the waves spend 30 % or more of their cycles parked
    on s_waitcnt (SQ_WAIT_ANY), the kernel is latency-bound: dependent node fetches with too few
    waves to cover them, the busiest unit listed beside it."""
    if not pmc or "valu_insts" not in pmc:
        return None
    cyc = kernel_ms * 1e-3 * CLOCK_GHZ * 1e9
    secs = kernel_ms * 1e-3
    busy = {"valu": pmc["valu_insts"] * VALU_CYC / (SIMDS * cyc),
            "salu": pmc.get("salu_insts", 0) / (CUS * cyc)}
    if "l2_request_bytes" in pmc:
        busy["l2"] = pmc["l2_request_bytes"] / secs / 1e9 / L2_PEAK_GBS
    if "traffic_bytes" in pmc:
        busy["hbm"] = pmc["traffic_bytes"] / secs / 1e9 / HBM_PEAK_GBS
    top = max(busy, key=busy.get)
    wait = pmc.get("wait_any_frac")
    bound = top if busy[top] >= 0.7 else ("latency" if wait is not None and wait >= 0.3 else top)
    return {"bound": bound, "busy": {k: round(v, 4) for k, v in busy.items()},
            "wave_cycles": {"wait_any": wait, "wait_inst_any": pmc.get("wait_inst_any_frac"),
                            "active": pmc.get("active_frac")},
            "l1_hit_rate": pmc.get("l1_hit_rate"), "l2_hit_rate": pmc.get("l2_hit_rate"),
            "l2_request_bytes": pmc.get("l2_request_bytes"),
            "per_wave": {k: round(pmc[k + "_insts"] / max(1, pmc.get("waves", 1)), 1)
                         for k in ("valu", "salu", "vmem_rd", "vmem_wr", "lds", "branch") if k + "_insts" in pmc},
            "source": pmc.get("source")}


def roofline(kernel, algo_bytes, kernel_ms, pmc):
    """Dominant kernel's roofline.  `bound` is measured (limiter(): the busiest unit from the
    kernel's counters, or "latency" when no unit is half busy and the waves mostly wait on
    memory).  `achieved` = algorithmic bytes / average launch time, priced against the peak of
    the level that serves those bytes -- HBM when the counter-measured HBM traffic is at
    least half the algorithmic bytes, else the L2 aggregate (the scene's nodes and triangles
    are re-read from the caches); that fraction is a secondary figure (`frac_basis`)."""
    secs = kernel_ms * 1e-3
    achieved = algo_bytes / secs / 1e9
    traffic = pmc["traffic_bytes"] if pmc and "traffic_bytes" in pmc else None
    hbm_gbs = traffic / secs / 1e9 if traffic is not None else None
    serves_hbm = traffic is not None and traffic >= 0.5 * algo_bytes
    peak = HBM_PEAK_GBS if serves_hbm else L2_PEAK_GBS
    lim = limiter(pmc, kernel_ms)
    r = {"bound": lim["bound"] if lim else ("hbm" if serves_hbm else "l2"), "achieved": round(achieved, 1),
         "peak": peak, "unit": "GB/s", "frac": round(achieved / peak, 4),
         "frac_basis": ("algorithmic bytes (SURVEY 8d) / " + ("HBM" if serves_hbm else "L2 aggregate") +
                        " peak -- secondary; the measured limiter is `bound` / `limiter`"),
         "traffic": traffic, "kernel": kernel, "kernel_ms": round(kernel_ms, 4),
         "algo_bytes_per_launch": int(algo_bytes),
         "hbm_gbs_measured": round(hbm_gbs, 1) if hbm_gbs is not None else None,
         "hbm_frac_measured": round(hbm_gbs / HBM_PEAK_GBS, 4) if hbm_gbs is not None else None,
         "l2_frac": round(achieved / L2_PEAK_GBS, 4)}
    if lim:
        r["limiter"] = lim
    if pmc:
        r["traffic_source"] = pmc["source"]
        if "l2_hit_rate" in pmc:
            r["l2_hit_rate"] = pmc["l2_hit_rate"]
    return r


def part_scaling(reps, torch, seed, steps, value, frame_s, counts=(2, 4, 8)):
    """The N-GPU frame on one GPU: every part r of N (its 8-row bands, multigpu.py part_runs,
    multigpu.py) rendered alone, with the same frames in flight as the headline steps
    (`reps`: the replicas the steps rotate over).  With one GPU per part the N-GPU node takes
    the slowest part's time per frame, so the predicted strong-scaling efficiency is
    frame / (N x max part) -- band imbalance, launch latency and the tail of a small grid all
    show up in it (main.cpp:38-39 deals row bands to threads the same way)."""
    out = {}
    F = len(reps)
    for n in counts:
        ms = [0.0] * n
        issue = [0.0] * n
        order = range(n - 1, -1, -1) if os.environ.get("RTG_BENCH_PARTS_REVERSED") else range(n)
        for r in order:
            def step(k, r=r, n=n):
                ds_, h, l, sp = reps[k % F]
                ds_.render_device(h.data_ptr(), l.data_ptr(), sp, seed=seed, part=(r, n))
            # warm-up: every replica renders this part once (its tile map for the part's rows is
            # built on first use)
            e, _ = measure(step, torch, steps, F, lambda: None, serial=lambda: None)
            ms[r] = e / steps * 1e3
            issue[r] = measure.issue_s / steps * 1e3
        worst = max(ms)
        out[str(n)] = {"part_ms": [round(x, 4) for x in ms], "max_part_ms": round(worst, 4),
                       "issue_ms": [round(x, 4) for x in issue],
                       "predicted_efficiency": round(frame_s * 1e3 / (n * worst), 4),
                       "predicted_mrays_s": round(value * frame_s * 1e3 / worst, 1)}
        log(f"parts x{n}: max part {worst:.4f} ms, predicted efficiency {out[str(n)]['predicted_efficiency']}")
    return out


def frame_stats(ds, torch, render_counting, reduce_sum):
    ds.reset_stats()
    render_counting()
    torch.cuda.synchronize()
    st = reduce_sum(ds.stats())
    return st, st["camera_rays"] + st["secondary_rays"] + st["shadow_rays"]


def sweep_point(args, torch, rtgpu, local, K, hdr, ldr):
    """One K of the sweep on this GPU: rays, Mrays/s, dominant kernel and its roofline."""
    sub = tempfile.mkdtemp(prefix="rtg_sweep_")
    old = os.getcwd()
    try:
        xml, _ = make_workload(args, sub, K=K)
        os.chdir(sub)
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, local)
        sptr = torch.cuda.current_stream().cuda_stream
        st, rays = frame_stats(ds, torch, lambda: ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr,
                                                                   flags=rtgpu.RTG_RENDER_COUNT_STATS), lambda s: s)
        steps = max(5, args.steps // 2)
        e, _ = measure(lambda: ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr), torch, steps, 1, lambda: None)
        kt = kernel_times(ds, torch, lambda: ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr,
                                                              flags=rtgpu.RTG_RENDER_TIMING), 5)
        kb = kernel_bytes(st, args.width, args.height)
        dom = max((k for k in kt if k in kb), key=lambda k: kt[k])
        rl = roofline(dom, kb[dom], kt[dom], pmc_summary(dom, K, 1))
        ds.close()
        hs.close()
        return {"mrays_s": round(rays * steps / e / 1e6, 1), "ms_per_frame": round(e / steps * 1e3, 4),
                "rays": int(rays), "kernels_ms": {k: round(v, 4) for k, v in kt.items()}, "roofline": rl,
                "mode": "serial (one stream, one frame at a time)"}
    finally:
        os.chdir(old)
        shutil.rmtree(sub, ignore_errors=True)


def main():
    args = parse()
    import torch

    import multigpu
    import rtgpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with "
                         "torch.distributed.run --nproc-per-node N (one rank per GPU)")
    dist = None
    # RTG_BENCH_BACKEND=gloo: rehearse the multi-rank flow on a box with fewer GPUs than ranks
    # (ranks share devices round-robin); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("RTG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    barrier = (lambda: dist.barrier()) if dist else (lambda: None)
    rdev = f"cuda:{local}" if backend == "nccl" else "cpu"

    def reduce_max(x):
        if not dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def reduce_sum(stats):
        if not dist:
            return stats
        keys = sorted(stats)
        t = torch.tensor([stats[k] for k in keys], dtype=torch.float64, device=rdev)
        dist.all_reduce(t)
        return {k: int(v) for k, v in zip(keys, t.tolist())}

    tmp = tempfile.mkdtemp(prefix=f"rtg_bench_r{rank}_")
    old = os.getcwd()
    frame = None
    try:
        xml, desc = make_workload(args, tmp)
        os.chdir(tmp)
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, local)
        cam = hs.camera(0)
        H, W = cam["height"], cam["width"]
        hdr = torch.empty((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")
        ldr = torch.empty((H, W, 3), dtype=torch.uint8, device=f"cuda:{local}")
        seed = 0x5EED
        part = (rank, world)
        sptr = torch.cuda.current_stream().cuda_stream

        def render(flags=0):
            ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr, seed=seed, flags=flags, part=part)

        # frames in flight: replicas 1..F-1 of the scene, each with its own frame buffers and
        # stream; step k renders frame k on replica k % F (replica 0 = ds, on a stream of its
        # own when F > 1 -- not torch's current stream, which the serial and counting passes use)
        # (C5's 4K x 64 spp frames fill the GPU on their own and its ray-tree levels take ~10 GB
        # per replica: one; the others 8 -- C3 1 892 -> 4 153 Mrays/s, C4 1 653 -> 2 102, C2
        # 7 792 -> 14 083: a frame's slowest waves no longer idle the GPU, profiles/r03v)
        F = args.inflight or (1 if args.config == "c5" else FRAMES_IN_FLIGHT)
        streams = [torch.cuda.Stream() for _ in range(F if F > 1 else 0)]
        reps = [(ds, hdr, ldr, streams[0].cuda_stream if F > 1 else sptr)]
        for k in range(1, F):
            reps.append((rtgpu.DeviceScene(hs, local), torch.empty_like(hdr), torch.empty_like(ldr),
                         streams[k].cuda_stream))

        def render_step(k):
            r, h, l, sp = reps[k % F]
            r.render_device(h.data_ptr(), l.data_ptr(), sp, seed=seed, part=part)

        # set-up: one render per replica (each allocates its work buffers on its first render)
        for k in range(F):
            render_step(k)
        torch.cuda.synchronize()

        # untimed counting pass: rays / BVH nodes / triangle tests of the whole frame
        log(f"scene ready: {hs.counts()}, part {rank}/{world}, counting pass")
        part_st, part_rays = frame_stats(ds, torch, lambda: render(rtgpu.RTG_RENDER_COUNT_STATS), lambda s: s)
        st = reduce_sum(part_st)
        rays = st["camera_rays"] + st["secondary_rays"] + st["shadow_rays"]

        log(f"rays/frame {rays} (this part {part_rays}); timing {args.steps} steps, {F} frames in flight")
        elapsed, kern_ms = measure(render_step, torch, args.steps, args.warmup, barrier, serial=lambda: render())
        log(f"timed: {elapsed / args.steps * 1e3:.3f} ms/step")
        elapsed = reduce_max(elapsed)
        kern_ms = reduce_max(kern_ms)
        value = rays * args.steps / elapsed / 1e6
        # the same frames one after another on one stream (no overlap): the single-frame rate
        s_el, _ = measure(lambda: render(), torch, args.steps, 1, barrier)
        s_el = reduce_max(s_el)

        ktimes = kernel_times(ds, torch, lambda: render(rtgpu.RTG_RENDER_TIMING), args.steps)
        # the library times the kernels of the last pass (its samples: several per pass in the
        # wavefront and ray-tree pipelines): bytes of this rank's pass
        pass_samples = ds.timed_samples()
        kbytes = {k: v * pass_samples / max(1, cam["spp"]) for k, v in kernel_bytes(part_st, W, H).items()}
        dom = max((k for k in ktimes if k in kbytes), key=lambda k: ktimes[k])
        K = int(args.K) if args.config == "headline" else None
        share = part_rays / max(rays, 1)
        rl = roofline(dom, kbytes[dom], ktimes[dom], pmc_summary(dom, K, world, share, workload=args.config))
        rl.update({"kernels_ms": {k: round(v, 4) for k, v in ktimes.items()}, "frame_ms": round(kern_ms, 4),
                   "frame_algo_bytes": int(kernel_bytes(st, W, H)["frame"]),
                   "frame_l2_frac": round(kernel_bytes(st, W, H)["frame"] / (kern_ms * 1e-3) / 1e9 / L2_PEAK_GBS, 4)})
        ext = max(rays - st["shadow_rays"], 1)
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded procedural height field, written as the reference's XML+PLY)",
            "config": {
                "workload": desc,
                "scene_K": K if K else int(hs.counts()["faces"]),
                "width": W, "height": H, "spp": int(cam["spp"]),
                "rays_per_frame": int(rays),
                "camera_rays": int(st["camera_rays"]), "shadow_rays": int(st["shadow_rays"]),
                "node_visits_per_extend_ray": round(st["node_visits"] / ext, 2),
                "tri_tests_per_extend_ray": round(st["tri_tests"] / ext, 2),
                "shadow_node_visits_per_ray": round(st["shadow_node_visits"] / max(st["shadow_rays"], 1), 2),
                "shadow_wide_node_visits_per_ray": round(st.get("shadow_wide_visits", 0) / max(st["shadow_rays"], 1), 2),
                "shadow_fallback_rays": int(st.get("shadow_fallbacks", 0)),
                "shadow_tri_tests_per_ray": round(st["shadow_tri_tests"] / max(st["shadow_rays"], 1), 2),
                "parallelism": f"image partition x{world}: 8-row bands dealt round-robin rotated one slot per round, rank r "
                               f"renders band k*{world} + ((r - k) mod {world}) (one frame per step)",
                "frames_in_flight": F,
                "serial": {"ms_per_step": round(s_el / args.steps * 1e3, 4),
                           "mrays_s": round(rays * args.steps / s_el / 1e6, 2),
                           "what": "the same steps issued on one stream, each frame after the previous one"},
            },
            "roofline": rl,
            "cpu_baseline": None,
        }

        if not args.no_extras:
            # host framebuffer gather: every rank renders its rows straight into one page-locked
            # shared frame (LDR = what main.cpp saves; + the float frame for a tonemapped camera)
            name = f"rtg_bench_{os.environ.get('MASTER_PORT', str(os.getpid()))}"
            if rank == 0:
                frame = multigpu.SharedFrame(name, H, W, hdr=cam["tonemapped"], ldr=True, create=True)
            barrier()
            if rank != 0:
                frame = multigpu.SharedFrame(name, H, W, hdr=cam["tonemapped"], ldr=True)
            frame.pin()
            fr = frame
            g_el, _ = measure(lambda: multigpu.render_part(ds, rank, world, hdr.data_ptr(), ldr.data_ptr(), sptr, fr,
                                                           seed=seed), torch, args.steps, 1, barrier)
            g_el = reduce_max(g_el)
            result["gather"] = {"ms_per_frame": round(g_el / args.steps * 1e3, 4),
                                "mrays_s": round(rays * args.steps / g_el / 1e6, 2),
                                "bytes_per_frame": int(H * W * 3 * (5 if cam["tonemapped"] else 1)),
                                "what": "rtg_render of each rank's part straight into one page-locked /dev/shm frame "
                                        "(the kernels write the pixels over the bus, no copy after the render; "
                                        "multigpu.render_part)"}
            if world == 1:
                # the drop-in host path (rtg_render: per-scene stream, page-locked frame, as the CLI)
                ph = rtgpu.PinnedArray((H, W, 3), "float32") if cam["tonemapped"] else None
                pl = rtgpu.PinnedArray((H, W, 3), "uint8")
                outs = (ph.array if ph else None, pl.array)
                for _ in range(2):
                    ds.render(0, seed=seed, out=outs)
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    ds.render(0, seed=seed, out=outs)
                hf = (time.perf_counter() - t0) / args.steps
                t0 = time.perf_counter()
                rtgpu.write_png(os.path.join(tmp, "frame.png"), pl.array)
                png = time.perf_counter() - t0
                result["host_frame"] = {"render_ms": round(hf * 1e3, 4), "png_ms": round(png * 1e3, 2),
                                        "mrays_s": round(rays / hf / 1e6, 2),
                                        "what": "rtg_render into page-locked host frames (CLI path; the PNG "
                                                "encode of main.cpp:197 timed apart)"}
                pl.close()
                if ph:
                    ph.close()
            if world == 1:
                # at least 20 frames per replica per part: the steady state of F frames in flight
                # (a short run is dominated by filling and draining the streams)
                result["parts"] = part_scaling(reps, torch, seed, max(args.steps, 20 * F), value,
                                               elapsed / args.steps)
            if world == 1:
                # opt-in ordered closest hit (RTG_RENDER_ORDERED): same frame, its agreement with
                # the reference-order walk measured here (pixels whose float bits differ)
                torch.cuda.synchronize()
                ref_hdr = hdr.clone()
                render(rtgpu.RTG_RENDER_ORDERED)
                torch.cuda.synchronize()
                n_fail = int((hdr.view(torch.int32) != ref_hdr.view(torch.int32)).any(dim=2).sum().item())
                o_st, o_rays = frame_stats(ds, torch, lambda: render(rtgpu.RTG_RENDER_ORDERED | rtgpu.RTG_RENDER_COUNT_STATS),
                                           lambda s: s)
                o_el, _ = measure(lambda: render(rtgpu.RTG_RENDER_ORDERED), torch, args.steps, 1, barrier)
                o_kt = kernel_times(ds, torch, lambda: render(rtgpu.RTG_RENDER_ORDERED | rtgpu.RTG_RENDER_TIMING),
                                    args.steps)
                result["ordered"] = {
                    "mrays_s": round(o_rays * args.steps / o_el / 1e6, 2),
                    "ms_per_frame": round(o_el / args.steps * 1e3, 4),
                    "kernels_ms": {k: round(v, 4) for k, v in o_kt.items()},
                    "n_fail_pixels": n_fail, "pixels": int(H * W),
                    "wide_visits_per_camera_ray": round(o_st["extend_wide_visits"] / max(o_st["camera_rays"], 1), 2),
                    "checked_out_rays": int(o_st["extend_fallbacks"]),
                    "what": "opt-in RTG_RENDER_ORDERED: camera rays walk the 4-wide BVH nearest child first with a "
                            "checked (t, object, face) minimum, the reference walk where the check fails; "
                            "not the headline value (agreement measured, not proven)"}

        if rank == 0 and world == 1 and not args.no_sweep and args.config == "headline":
            sweep = {}
            for Ks in SWEEP_K:
                if Ks == args.K:
                    ser = result["config"]["serial"]
                    sweep[str(Ks)] = {"mrays_s": ser["mrays_s"], "ms_per_frame": ser["ms_per_step"],
                                      "rays": int(rays), "kernels_ms": rl["kernels_ms"],
                                      "roofline": {k: rl[k] for k in rl if k not in ("kernels_ms",)},
                                      "mode": "serial (one stream, one frame at a time)"}
                    continue
                log(f"sweep K={Ks}")
                sweep[str(Ks)] = sweep_point(args, torch, rtgpu, local, Ks, hdr, ldr)
            result["sweep_K"] = sweep
        # the reference's CPU path on this host, rank 0 only, outside the timed region, at every N
        # (the same frame or row band: its rate does not depend on how the GPUs split it); the
        # rays of the rows it renders from this GPU's counting render of those rows
        if rank == 0 and not args.no_cpu_baseline:
            def count_rays(r0, r1):
                if (r0, r1) == (0, H) and world == 1:
                    return rays
                ds.reset_stats()
                ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr, seed=seed, rows=(r0, r1),
                                 flags=rtgpu.RTG_RENDER_COUNT_STATS)
                torch.cuda.synchronize()
                s_ = ds.stats()
                return s_["camera_rays"] + s_["secondary_rays"] + s_["shadow_rays"]
            cs = CPU_SAMPLE.get(args.config, {})
            result["cpu_baseline"] = cpu_baseline(tmp, xml, count_rays, cs.get("reps", args.cpu_reps),
                                                  rows=cs.get("rows"), kind=cs.get("kind"))
        if rank == 0:
            print(json.dumps(result), flush=True)
        barrier()     # the other ranks wait for rank 0's CPU leg before tearing the group down
    finally:
        if frame is not None:
            frame.close()
        os.chdir(old)
        shutil.rmtree(tmp, ignore_errors=True)
        if dist:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
