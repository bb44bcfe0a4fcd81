"""Summarise rocprofv3 outputs under gpurun_out/prof into committed profiles/ files.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM / rocprofv3 section):
FETCH_SIZE and WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half of the
bytes of a coalesced streaming read, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

    python tools/summarize_prof.py --round r01
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
OUT = os.path.join(ROOT, "profiles")

WORK = {  # workload -> (kernel substring, algorithmic bytes per launch, note)
    "fkjac32": ("k_fk<float, 8>", (8 + 12 + 48) * 4 * (1 << 20), "FK + 6x8 J, fp32, N = 2^20: 8 q in, 60 out"),
    "fkjac32t": ("k_fk<float, 8>", (8 + 12 + 48) * 4 * (1 << 20),
                 "FK + 6x8 J, fp32, N = 2^20, tiled SoA (tile as run), generic kernel"),
    "fkjac64t": ("k_fk<double, 8>", (8 + 12 + 48) * 8 * (1 << 20), "FK + 6x8 J, fp64, N = 2^20, tiled SoA (tile 4096)"),
    "fkjac32s": ("kinhip_jit_fk_f32", (8 + 12 + 48) * 4 * (1 << 20),
                 "FK + 6x8 J, fp32, N = 2^20, plain SoA rows padded by 256, plan-specialised kernel"),
    "fkjac32sjl": ("kinhip_jit_fk_f32", (8 + 12 + 48) * 4 * (1 << 20),
                   "FK + 6x8 J, fp32, N = 2^20, plain SoA rows with ld = N (the Julia shim's ROCMatrix(N, 8) / "
                   "ROCArray(N, 6, 8)), plan-specialised kernel (bench fk_jac_f32_julia_layout)"),
    "fkjac32ts": ("kinhip_jit_fk_f32", (8 + 12 + 48) * 4 * (1 << 20),
                  "FK + 6x8 J, fp32, N = 2^20, tiled SoA (tile 8192), plan-specialised kernel (bench headline)"),
    "fkjac32ts22": ("kinhip_jit_fk_f32", (8 + 12 + 48) * 4 * (1 << 22),
                    "FK + 6x8 J, fp32, N = 2^22 (4x the Infinity Cache), tiled SoA (tile 8192), specialised"),
    "fkjac32ts24": ("kinhip_jit_fk_f32", (8 + 12 + 48) * 4 * (1 << 24),
                    "FK + 6x8 J, fp32, N = 2^24 (16x the Infinity Cache), tiled SoA (tile 8192), specialised"),
    "collg32ts": ("kinhip_jit_coll_1_f32", (8 + 14 + 14 * 8) * 4 * (1 << 20),
                  "config 5 / IneqConst: 14 distances + 14x8 gradients, fp32, N = 2^20, tiled SoA (tile 8192), "
                  "specialised"),
    "fkjac64ts": ("kinhip_jit_fk_f64", (8 + 12 + 48) * 8 * (1 << 20),
                  "FK + 6x8 J, fp64, N = 2^20, tiled SoA (tile as run), plan-specialised kernel"),
    "fk6_64ts": ("kinhip_jit_fk_f64", (8 + 72) * 8 * (1 << 20),
                 "FK of 6 links (config 2), fp64, N = 2^20, tiled SoA (tile 4096), plan-specialised kernel"),
    "ik32s": ("kinhip_jit_ik_6_", 65536 * (12 + 8 + 8 + 1 + 2) * 4,
              "config 4: DLS IK, 65,536 targets, 64 iterations, 3 restarts, fp32, plan-specialised kernels; one solve "
              "= the two-phase schedule's two launches (ik_6_1: attempt 0 of every target, G = 1; ik_6_4: the other "
              "attempts of the unsolved targets, G = 4), counters and durations summed over both"),
    "coll32s": ("kinhip_jit_coll_0_f32", (8 + 1) * 4 * (1 << 20),
                "config 5 validity: FK + 14 spheres vs 7-box fridge SDF, min distance, fp32, N = 2^20, specialised"),
    "collg32s": ("kinhip_jit_coll_1_f32", (8 + 14 + 14 * 8) * 4 * (1 << 20),
                 "config 5 / IneqConst: 14 distances + 14x8 gradients, fp32, N = 2^20, specialised"),
    "scene32s": ("kinhip_jit_collc_1_f32", ((8 + 4) + 14 + 14 * 8 + 1) * 4 * (1 << 20),
                 "f2 door sweep (bench f2_scene_door_sweep): boxes attached to the fridge, one door angle per sample, "
                 "14 distances + 14x8 gradients + the minimum, fp32, N = 2^20, scene-specialised kernel (round 6: "
                 "kin_plan_specialize_scene, the fridge's tables compiled in; rounds 3-5: kinhip_jit_colls_1_2)"),
    "cik32s": ("kinhip_jit_ikt_6_", 4096 * (12 + 8 + 8 + 1 + 3) * 4,
               "f3 stage 2 (bench f3_collision_ik): kin_ik_coll_batch of 4,096 fridge targets from stage 1's answers, "
               "128 iterations, 3 restarts side by side in 4 lane groups of 16 sphere lanes, fp32, specialised"),
    "cikp32s": ("kinhip_jit_ikt_6_", 4096 * (12 + 8 + 8 + 1 + 3) * 4,
                "bench f3_collision_ik_pillar_4096: stage 2 of 4,096 targets around a pillar on the elbow (most "
                "stage-1 answers collide), 128 iterations, 3 restarts, fp32, specialised"),
    "fkjac64": ("k_fk<double, 8>", (8 + 12 + 48) * 8 * (1 << 20), "FK + 6x8 J, fp64, N = 2^20"),
    "fk6_64": ("k_fk<double, 8>", (8 + 72) * 8 * (1 << 20), "FK of 6 links (config 2), fp64, N = 2^20"),
    "ik32": ("k_ik_dls<float, 8, 6, 4>", 65536 * (12 + 8 + 8 + 1 + 2) * 4,
             "config 4: DLS IK, 65,536 targets, 64 iterations, 3 restarts, G = 4 lanes per target, fp32"),
    "coll32": ("k_coll<float, 8, false>", (8 + 1) * 4 * (1 << 20),
               "config 5 validity: FK + 14 spheres vs 7-box fridge SDF, min distance out, fp32, N = 2^20"),
    "collg32": ("k_coll<float, 8, true>", (8 + 14 + 14 * 8) * 4 * (1 << 20),
                "config 5 / IneqConst: 14 distances + 14x8 gradients out, fp32, N = 2^20"),
}
N_CU, N_SIMD = 256, 4


def valu_metrics(c):
    """VALU utilisation from the SQ counters (MI355X_MICROARCH.md: SQ_* cycle counters count
    quad-cycles per wave; GRBM_GUI_ACTIVE is summed over the 8 XCDs).

    valu_busy = issued VALU instructions x 2 cycles (a wave64 fp32 VALU instruction occupies a SIMD
    for 2 cycles) / (SIMD count x elapsed cycles): the fraction of SIMD cycles spent issuing VALU
    work.  It cannot exceed 1 while the elapsed-cycle estimate is right; transcendental and fp64
    instructions take more than 2 cycles, so for them it is a lower bound.
    The earlier figure, SQ_ACTIVE_INST_VALU x 4 / (SIMDs x cycles), is kept as
    `sq_active_inst_valu_ratio`: that counter sums, over waves, the cycles during which each wave has
    a VALU instruction in flight, and the in-flight cycles of co-resident waves on one SIMD overlap,
    so the ratio is not a utilisation (it reached 1.10 on the collision kernel)."""
    if "GRBM_GUI_ACTIVE" not in c:
        return {}
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    out = {"elapsed_cycles": cyc}
    if "SQ_INSTS_VALU" in c:
        out["valu_busy"] = c["SQ_INSTS_VALU"] * 2 / (N_CU * N_SIMD) / cyc
        if "SQ_WAVES" in c:
            out["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
    if "SQ_ACTIVE_INST_VALU" in c:
        out["sq_active_inst_valu_ratio"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (N_CU * N_SIMD) / cyc
    return out


def mem_metrics(c):
    """Memory-side backpressure and address translation (TCC / TCP counters, when collected):
    write-credit stall cycles of the L2 -> memory path per elapsed cycle (summed over the 16 TCC
    channels of each XCD, so a rate of 1 means one channel stalled all the time on average per XCD),
    and the UTCL1 (per-CU TLB) miss fraction."""
    out = {}
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
    for k in ("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "TCC_EA0_WRREQ_STALL_sum"):
        if k in c:
            out[k] = c[k]
            if cyc:
                out[k.replace("_sum", "_per_cycle")] = c[k] / cyc
    if "TCP_UTCL1_TRANSLATION_MISS_sum" in c and "TCP_UTCL1_REQUEST_sum" in c:
        out["utcl1_requests"] = c["TCP_UTCL1_REQUEST_sum"]
        out["utcl1_misses"] = c["TCP_UTCL1_TRANSLATION_MISS_sum"]
        out["utcl1_miss_frac"] = c["TCP_UTCL1_TRANSLATION_MISS_sum"] / max(1.0, c["TCP_UTCL1_REQUEST_sum"])
    return out


def recompute(paths):
    """Rewrite the `valu` block of committed PMC summaries from their stored SQ / GRBM counters."""
    for p in paths:
        with open(p) as f:
            d = json.load(f)
        if not d.get("sq"):
            continue
        d["valu"] = valu_metrics(d["sq"])
        d["valu_note"] = "valu block recomputed by tools/summarize_prof.py --recompute (issue-based valu_busy)"
        with open(p, "w") as f:
            json.dump(d, f, indent=1)
        print(os.path.basename(p), {k: round(v, 3) for k, v in d["valu"].items() if k != "elapsed_cycles"})


def counters(tag):
    """Per-launch mean of each counter per matching kernel, summed over the matching kernels (a
    workload whose one unit of work is several launches, e.g. the two-phase IK solve)."""
    agg = collections.defaultdict(list)
    kern = WORK[tag][0]
    for f in glob.glob(os.path.join(PROF, f"{tag}_*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = collections.defaultdict(float)
    for (_, k), v in agg.items():
        out[k] += sum(v) / len(v)
    return dict(out)


def stats(path, kern):
    """Kernel-stats row of the matching kernel; several matching kernels (one unit of work = several
    launches) are summed: AverageNs = the sum of their average durations."""
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Name"]]
    if not rows:
        return None
    if len(rows) == 1:
        return {k: rows[0][k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "StdDev")}
    return {"Name": " + ".join(r["Name"] for r in rows), "Calls": rows[0]["Calls"],
            "AverageNs": str(sum(float(r["AverageNs"]) for r in rows)),
            "per_kernel_avg_ns": {r["Name"]: float(r["AverageNs"]) for r in rows}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--recompute", nargs="*", help="rewrite the valu block of these profiles/*_pmc_*.json files")
    a = ap.parse_args()
    if a.recompute is not None:
        recompute(a.recompute or sorted(glob.glob(os.path.join(OUT, "*pmc_*.json"))))
        return
    os.makedirs(OUT, exist_ok=True)
    for tag, (kern, alg, note) in WORK.items():
        c = counters(tag)
        if not c:
            continue
        st = None
        for p in glob.glob(os.path.join(PROF, f"{tag}_trace", "*_kernel_stats.csv")):
            st = stats(p, kern)
            shutil.copy(p, os.path.join(OUT, f"{a.round}_{tag}_kernel_stats.csv"))
        hbm = None
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        d = {"workload": tag, "note": note, "kernel": kern, "round": a.round,
             "algorithmic_bytes_per_launch": alg, "hbm_bytes_per_launch": hbm,
             "traffic_over_algorithmic": (hbm / alg) if hbm else None,
             "fetch_size_kb_raw": c.get("FETCH_SIZE"), "write_size_kb": c.get("WRITE_SIZE"),
             "avg_duration_ns_trace": float(st["AverageNs"]) if st else None,
             "per_kernel_avg_ns": st.get("per_kernel_avg_ns") if st else None,
             "achieved_GBs_trace": (alg / float(st["AverageNs"])) if st else None,
             "sq": {k: v for k, v in c.items() if k.startswith(("SQ_", "GRBM_"))},
             "valu": valu_metrics(c),
             "memory_side": mem_metrics(c),
             "method": "rocprofv3 --kernel-trace --stats, then separate --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ_*), "
                       "20 launches each via tools/prof_kernel.py; hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950)"}
        with open(os.path.join(OUT, f"{a.round}_pmc_{tag}.json"), "w") as f:
            json.dump(d, f, indent=1)
        # the headline kernel's and the fp64 leg's PMC passes, read by bench.py (roofline.traffic)
        for t_, fn in (("fkjac32ts", "pmc_fk_jac_f32.json"), ("fkjac64ts", "pmc_fk_jac_f64.json")):
            if tag == t_:
                with open(os.path.join(OUT, fn), "w") as f:
                    json.dump(d, f, indent=1)
        print(json.dumps({k: d[k] for k in ("workload", "hbm_bytes_per_launch", "traffic_over_algorithmic",
                                            "avg_duration_ns_trace", "achieved_GBs_trace")}))
    b = os.path.join(PROF, "bench", "bench_kernel_stats.csv")
    if os.path.exists(b):
        shutil.copy(b, os.path.join(OUT, f"{a.round}_bench_kernel_stats.csv"))
        print("bench:", stats(b, "kinhip_jit_fk_f32"))


if __name__ == "__main__":
    main()
