"""Headline bench: Mrays/s on the BASELINE.json synthetic K-triangle scene at 1920x1080
(primary + shadow rays), with the HBM-roofline fraction of the render kernel and the
reference's own multithreaded CPU path timed on this host beside it.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one full 1920x1080 frame (one sample pass) traced and shaded on each rank,
inputs (scene, BVH) resident in HBM.  Ranks are independent (sample-parallel: rank r
traces sample pass r of the same frame) -> weak scaling, no collective on the data path;
the only collectives are the barriers around the timed region and the max-over-ranks of
the elapsed time.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "advanced-cpu-raytracing_amd")
sys.path.insert(0, PKG)

METRIC = "Mrays/sec + achieved HBM GB/s fraction, 1920×1080 primary+shadow rays"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--K", type=int, default=100352, help="triangles in the synthetic height field")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=8, help="reference THREAD_COUNT (main.cpp:15)")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--sweep", action="store_true", help="also report K in {1k,10k,1M} (extra field)")
    p.add_argument("--config", default="headline", choices=["headline", "c2", "c3", "c4", "c5"],
                   help="BASELINE.json configuration (c2-c5: one frame = all camera samples)")
    return p.parse_args()


CONFIG_DESC = {
    "c2": "C2 conductor Cornell box + OriginalPhong BRDF, 800x800, 1 spp, depth 6",
    "c3": "C3 70k-triangle mesh + area light, OriginalBlinnPhong, 1920x1080, 4 spp",
    "c4": "C4 10k-triangle tree x 100 MeshInstances (~1M effective) + spherical env light, "
          "TorranceSparrow kdfresnel, 1920x1080, 16 spp",
    "c5": "C5 870k-triangle dielectric mesh + mirror sphere + Perlin ground, depth 5, 3840x2160, 64 spp",
}


def make_workload(args, out_dir):
    import scenes
    if args.config == "headline":
        xml = scenes.synthetic_heightfield(out_dir, K=args.K, width=args.width, height=args.height)
        desc = (f"synthetic height field K={args.K} tris, {args.width}x{args.height}, 1 spp, 1 point light, "
                "default Blinn-Phong, primary+shadow rays")
        return xml, desc
    if args.config == "c2":
        xml = scenes.config_c2(out_dir, os.path.join(ROOT, "tests", "golden", "scenes", "cornell_conductors.xml"))
    else:
        xml = getattr(scenes, "config_" + args.config)(out_dir)
    return xml, CONFIG_DESC[args.config]


def cpu_baseline(xml_dir, xml, rays_per_frame, threads, reps):
    """Reference CPU path (oracle/_ref/refdriver: the reference's own sources, row-band
    threads exactly as main.cpp:38-39,164-185) on this host; falls back to the oracle
    restatement ("port") when the reference build is absent."""
    drv = os.path.join(ROOT, "oracle", "_ref", "refdriver")
    sample = f"full 1920x1080 frame x {reps} reps, {threads} threads (render only: spawn->join)"
    if os.path.exists(drv):
        out = subprocess.run([drv, "bench", os.path.basename(xml), str(threads), str(reps)], cwd=xml_dir,
                             capture_output=True, text=True, timeout=600, check=True).stdout
        line = [l for l in out.splitlines() if l.startswith("{")][-1]
        secs = sorted(json.loads(line)["seconds"])
        med = secs[len(secs) // 2]
        return {"value": round(rays_per_frame / med / 1e6, 3), "unit": "Mrays/s", "cores": threads,
                "kind": "reference", "sample": sample, "seconds_median": round(med, 4)}
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob
    import rtgpu
    hs = rtgpu.HostScene(xml)
    secs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ob.render(hs, threads=threads)
        secs.append(time.perf_counter() - t0)
    secs.sort()
    med = secs[len(secs) // 2]
    return {"value": round(rays_per_frame / med / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": sample, "seconds_median": round(med, 4)}


def log(msg):
    """Progress on stderr (long configurations: keeps the run visibly alive)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def measure(ds, torch, hdr, ldr, steps, warmup, seed, barrier):
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    for k in range(warmup):
        ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr, seed=seed)
        torch.cuda.synchronize()
        log(f"warmup {k + 1}/{warmup}")
    torch.cuda.synchronize()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        starts[k].record(stream)
        ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr, seed=seed)
        ends[k].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / steps
    return elapsed, kern_ms


def kernel_times(ds, torch, hdr, ldr, steps, seed):
    """Per-kernel durations: HIP events recorded by the library around each kernel on the
    render's stream (RTG_RENDER_TIMING), averaged over `steps` frames run after the timed
    region."""
    import rtgpu
    sptr = torch.cuda.current_stream().cuda_stream
    acc = {}
    for _ in range(steps):
        ds.render_device(hdr.data_ptr(), ldr.data_ptr(), sptr, seed=seed, flags=rtgpu.RTG_RENDER_TIMING)
        for k, v in ds.timings().items():
            acc[k] = acc.get(k, 0.0) + v
    return {k: v / steps for k, v in acc.items()}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc.json, made by tools/pmc_summary.py from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    if not files:
        return None, None
    k = json.load(open(files[-1]))["kernels"].get(kernel + "<false>")
    return (k["traffic_bytes"] if k else None), os.path.basename(files[-1])


def kernel_bytes(st, W, H):
    """Algorithmic HBM bytes per launch of each kernel (32 B per node visit,
    36 B per triangle test, 64 B per ray = ray in + hit out, 15 B per pixel written)."""
    ext_rays = st["camera_rays"] + st["secondary_rays"]
    ext = 32 * st["node_visits"] + 36 * st["tri_tests"] + 64 * ext_rays
    shd = 32 * st["shadow_node_visits"] + 36 * st["shadow_tri_tests"] + 64 * st["shadow_rays"]
    return {"k_primary": ext, "k_shadow": shd, "k_render": ext + shd + 15 * W * H,
            "tree_levels": ext + shd, "frame": ext + shd + 15 * W * H}


def main():
    args = parse()
    import torch

    import rtgpu
    import scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # RTG_BENCH_BACKEND=gloo: rehearse the multi-rank flow on a box with fewer GPUs than ranks
    # (ranks share devices round-robin); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("RTG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    barrier = (lambda: dist.barrier()) if dist else (lambda: None)

    tmp = tempfile.mkdtemp(prefix=f"rtg_bench_r{rank}_")
    old = os.getcwd()
    try:
        xml, desc = make_workload(args, tmp)
        os.chdir(tmp)
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, local)
        cam = hs.camera(0)
        H, W = cam["height"], cam["width"]
        hdr = torch.empty((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")
        ldr = torch.empty((H, W, 3), dtype=torch.uint8, device=f"cuda:{local}")
        seed = 0x5EED + rank

        # untimed counting pass: rays / BVH nodes / triangle tests per frame
        log(f"scene ready: {hs.counts()}, counting pass")
        ds.reset_stats()
        ds.render_device(hdr.data_ptr(), ldr.data_ptr(), torch.cuda.current_stream().cuda_stream, seed=seed,
                         flags=rtgpu.RTG_RENDER_COUNT_STATS)
        torch.cuda.synchronize()
        st = ds.stats()
        rays = st["camera_rays"] + st["secondary_rays"] + st["shadow_rays"]

        log(f"rays/frame {rays}; timing {args.steps} steps")
        elapsed, kern_ms = measure(ds, torch, hdr, ldr, args.steps, args.warmup, seed, barrier)
        log(f"timed: {elapsed / args.steps * 1e3:.3f} ms/step")
        if dist:
            rdev = f"cuda:{local}" if backend == "nccl" else "cpu"
            t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            k = torch.tensor([kern_ms], dtype=torch.float64, device=rdev)
            dist.all_reduce(k, op=dist.ReduceOp.MAX)
            kern_ms = float(k.item())

        value = world * rays * args.steps / elapsed / 1e6
        ktimes = kernel_times(ds, torch, hdr, ldr, args.steps, seed)
        # the library times the kernels of the last sample pass: bytes of one pass
        kbytes = {k: v / max(1, cam["spp"]) for k, v in kernel_bytes(st, W, H).items()}
        # the dominant traversal kernel: k_primary (wavefront) or k_render (fused)
        dom = max((k for k in ktimes if k in kbytes), key=lambda k: ktimes[k])
        algo_bytes = kbytes[dom]
        achieved = algo_bytes / (ktimes[dom] * 1e-3) / 1e9
        frame_gbs = kbytes["frame"] * max(1, cam["spp"]) / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(dom) if args.config == "headline" else (None, None)
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded procedural height field, written as the reference's XML+PLY)",
            "config": {
                "workload": desc,
                "scene_K": int(args.K) if args.config == "headline" else int(hs.counts()["faces"]),
                "width": W, "height": H, "spp": int(cam["spp"]),
                "rays_per_frame": int(rays),
                "camera_rays": int(st["camera_rays"]), "shadow_rays": int(st["shadow_rays"]),
                "node_visits_per_extend_ray": round(st["node_visits"] / max(rays - st["shadow_rays"], 1), 2),
                "tri_tests_per_extend_ray": round(st["tri_tests"] / max(rays - st["shadow_rays"], 1), 2),
                "shadow_node_visits_per_ray": round(st["shadow_node_visits"] / max(st["shadow_rays"], 1), 2),
                "shadow_tri_tests_per_ray": round(st["shadow_tri_tests"] / max(st["shadow_rays"], 1), 2),
                "parallelism": f"sample-parallel x{world} (rank r traces sample pass r)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": dom,
                "kernel_ms": round(ktimes[dom], 4),
                "algo_bytes_per_launch": int(algo_bytes),
                "kernels_ms": {k: round(v, 4) for k, v in ktimes.items()},
                "frame_ms": round(kern_ms, 4),
                "frame_algo_bytes": int(kbytes["frame"] * max(1, cam["spp"])),
                "frame_frac": round(frame_gbs / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": None,
        }
        if args.sweep and rank == 0 and args.config == "headline":
            sweep = {}
            for K in (1000, 10082, 1002528):
                sub = tempfile.mkdtemp(prefix="rtg_sweep_")
                x2 = scenes.synthetic_heightfield(sub, K=K, width=W, height=H)
                os.chdir(sub)
                h2 = rtgpu.HostScene(x2)
                d2 = rtgpu.DeviceScene(h2, local)
                d2.reset_stats()
                d2.render_device(hdr.data_ptr(), ldr.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                 flags=rtgpu.RTG_RENDER_COUNT_STATS)
                torch.cuda.synchronize()
                s2 = d2.stats()
                r2 = s2["camera_rays"] + s2["shadow_rays"] + s2["secondary_rays"]
                e2, k2 = measure(d2, torch, hdr, ldr, max(3, args.steps // 2), 1, 0x5EED, lambda: None)
                sweep[str(K)] = {"mrays_s": round(r2 * max(3, args.steps // 2) / e2 / 1e6, 1),
                                 "kernel_ms": round(k2, 3), "rays": int(r2)}
                d2.close()
                h2.close()
                shutil.rmtree(sub, ignore_errors=True)
            result["sweep_K"] = sweep
        if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "headline":
            result["cpu_baseline"] = cpu_baseline(tmp, xml, rays, args.cpu_threads, args.cpu_reps)
        if rank == 0:
            print(json.dumps(result), flush=True)
    finally:
        os.chdir(old)
        shutil.rmtree(tmp, ignore_errors=True)
        if dist:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
