"""Per-kernel counters of one bench run's rocprofv3 --pmc passes (tools/gpu_r03.sh:
gpurun_out/<tag>/pmc*/run_counter_collection.csv, one pass per counter group), merged into the
summary bench.py reads (profiles/r*_pmc_K*.json): per kernel and launch

  read_bytes = 2 x FETCH_SIZE, write_bytes = WRITE_SIZE (KiB counters; the gfx950 FETCH
      correction of MI355X_MICROARCH.md), traffic_bytes = their sum (HBM);
  l2_hit_rate = TCC_HIT / (TCC_HIT + TCC_MISS); l2_requests = TCC_REQ, l2_request_bytes =
      128 B each (the L2 line);
  l1_hit_rate = 1 - TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES (vL1D);
  waves, valu / salu / vmem_rd / vmem_wr / lds / branch instructions (SQ_INSTS_*);
  wait_any / wait_inst_any / active fractions of SQ_WAVE_CYCLES (disjoint: parked on
      s_waitcnt or a barrier / issue-stalled / issuing).

bench.py turns the instruction counts into unit-busy fractions with its own live kernel time
(VALU: 2 cycles per wave64 instruction per SIMD; SALU: one scalar unit per CU) and picks the
roofline bound from them.  The fused k_shade instantiation (SH_FUSED) is named
k_shade_shadow, as the library's timing names it.

    python tools/pmc_kernels.py gpurun_out/<tag> [out.json] [--K K] [--gpus N]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def load(run_dir):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(os.path.join(run_dir, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(path)):
            m = re.search(r"rtg::(k_\w+)(<([^>]*)>)?", r["Kernel_Name"])
            if not m:
                continue
            base, targs = m.group(1), [t.strip() for t in (m.group(3) or "").split(",") if t.strip()]
            if base == "k_shade" and len(targs) >= 3 and targs[2] in ("2", "3"):
                # SH_FUSED / SH_FUSED_N: shading + shadow rays; with FRAME also the camera walk
                base = "k_frame" if len(targs) >= 6 and targs[5] == "true" else "k_shade_shadow"
            name = base + (f"<{targs[0]}>" if targs else "")
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return ({k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()},
            {k: {c: (sum(v), len(v)) for c, v in d.items()} for k, d in agg.items()})


# The library's timed stages (rtg_scene_timings) and the production kernels each one spans:
# a stage's counters are the sums over its kernels' launches in the run divided by the
# passes (launches of the stage's first kernel), i.e. per sample pass like its HIP-event time.
STAGES = {
    "k_primary": ("k_primary", "k_bigleaf", "k_hitfix", "k_refwalk"),
    "k_shadow": ("k_shadow", "k_shadow_one", "k_bigleaf_any", "k_shadow_fin", "k_shadow_fin_one"),
    "tree_levels": ("k_tree_gen", "k_tree_trace", "k_tree_shade", "k_shadow", "k_tree_scan", "k_tree_compact"),
}
EXTENSIVE = ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum",
             "TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum", "SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
             "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
             "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")


def stage_sums(totals, stage, tree):
    """Per-pass sums of a stage's production kernels (<false> / non-STATS instantiations);
    tree: the ray-tree pipeline's k_shadow belongs to tree_levels, not to a k_shadow stage."""
    members = STAGES[stage]
    names = [k for k in totals if k.split("<")[0] in members and "<true>" not in k]
    if not names:
        return None
    first = next((k for m in members for k in names if k.split("<")[0] == m), None)
    out = {}
    passes = 0
    for c in EXTENSIVE:
        vals = [totals[k][c][0] for k in names if c in totals[k]]
        if vals and c in totals[first]:
            n = totals[first][c][1]            # launches of the first kernel seen by this counter's pass(es)
            out[c] = sum(vals) / n
            passes = max(passes, n)
    return out, sorted(names), passes


def summarise(a):
    e = {}
    if "FETCH_SIZE" in a or "WRITE_SIZE" in a:
        rd, wr = 2.0 * a.get("FETCH_SIZE", 0.0) * 1024.0, a.get("WRITE_SIZE", 0.0) * 1024.0
        e.update(read_bytes=round(rd), write_bytes=round(wr), traffic_bytes=round(rd + wr))
    if "TCC_HIT_sum" in a and "TCC_MISS_sum" in a:
        e["l2_hit_rate"] = round(a["TCC_HIT_sum"] / max(1.0, a["TCC_HIT_sum"] + a["TCC_MISS_sum"]), 4)
    if "TCC_REQ_sum" in a:
        e["l2_requests"] = round(a["TCC_REQ_sum"])
        e["l2_request_bytes"] = round(a["TCC_REQ_sum"] * 128)
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in a and "TCP_TCC_READ_REQ_sum" in a:
        e["l1_hit_rate"] = round(1.0 - a["TCP_TCC_READ_REQ_sum"] / max(1.0, a["TCP_TOTAL_CACHE_ACCESSES_sum"]), 4)
        e["l1_accesses"] = round(a["TCP_TOTAL_CACHE_ACCESSES_sum"])
    for key, c in (("waves", "SQ_WAVES"), ("valu_insts", "SQ_INSTS_VALU"), ("salu_insts", "SQ_INSTS_SALU"),
                   ("vmem_rd_insts", "SQ_INSTS_VMEM_RD"), ("vmem_wr_insts", "SQ_INSTS_VMEM_WR"),
                   ("lds_insts", "SQ_INSTS_LDS"), ("branch_insts", "SQ_INSTS_BRANCH"),
                   ("smem_insts", "SQ_INSTS_SMEM"), ("wave_cycles_quad", "SQ_WAVE_CYCLES")):
        if c in a:
            e[key] = round(a[c])
    wc = a.get("SQ_WAVE_CYCLES")
    if wc:
        for key, c in (("wait_any_frac", "SQ_WAIT_ANY"), ("wait_inst_any_frac", "SQ_WAIT_INST_ANY"),
                       ("active_frac", "SQ_ACTIVE_INST_ANY")):
            if c in a:
                e[key] = round(a[c] / wc, 4)
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("out", nargs="?")
    ap.add_argument("--K", type=int, default=100352)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", default="headline", help="headline or a bench.py --config name (c3, c3ton, c4, c5)")
    a = ap.parse_args()
    res = {"note": "per launch; read = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE; l2_hit_rate = "
                   "TCC_HIT / (TCC_HIT + TCC_MISS); l1_hit_rate = 1 - TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES; "
                   "instruction counts SQ_INSTS_*; fractions of SQ_WAVE_CYCLES (tools/pmc_kernels.py)",
           "source": os.path.basename(os.path.normpath(a.run_dir)),
           "config": {"workload": a.workload, "K": a.K, "n_gpus": a.gpus},
           "kernels": {}}
    avg, totals = load(a.run_dir)
    res["kernels"] = {k: summarise(v) for k, v in sorted(avg.items())}
    tree = any(k.startswith("k_tree_trace") for k in totals)
    for stage in (("tree_levels",) if tree else ("k_primary", "k_shadow")):
        got = stage_sums(totals, stage, tree)
        if got:
            sums, names, passes = got
            e = summarise(sums)
            e.update(members=names, passes=passes, per="sample pass (sum over the stage's kernels)")
            res["kernels"]["stage:" + stage] = e
    for k, v in res["kernels"].items():
        print(k, json.dumps(v))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
