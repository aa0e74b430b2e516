#!/usr/bin/env python3
"""gpurun_out/prof_<workload>/ (scripts/profile.sh) -> profiles/<round>_<workload>_*.

Writes per workload:
  <round>_<w>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary, short kernel names
  <round>_<w>_pmc.csv           per-kernel average PMC values per launch
  <round>_<w>_kernel_resources.csv  per kernel: VGPR / AGPR / SGPR counts, LDS and scratch
                                bytes, workgroup and grid size of its first dispatch (VGPR as
                                rocprofv3 reports it on gfx950: half the compiler's granule-
                                rounded .vgpr_count, e.g. 48 for a 96-VGPR kernel)
and updates profiles/traffic.json with HBM bytes per launch of the bench's dominant kernel(s):
  bytes = 2 * FETCH_SIZE + WRITE_SIZE  (KB -> bytes).  FETCH_SIZE on gfx950 reports half the
  bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact for
  16-B stores; Infinity-Cache hits are counted in FETCH_SIZE.
usage: summarize_profiles.py <round> [workload ...]
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles")
TAS_PATH = ("tas_prep_kernel", "tas_eval_kernel")
GAS_PATH = ("gas_minfree_kernel", "gas_prep_kernel", "gas_rank_prep_kernel",
            "gas_rfit_single_kernel", "gas_rfit_closed_kernel", "gas_rfit_seq_kernel",
            "gas_fit_generic_kernel")


def short(name):
    m = re.search(r"(?:anonymous namespace\)::|pas::)(\w+)", name)
    if m:
        return m.group(1)
    if "rocprim" in name:
        kind = re.search(r"detail::(\w+?)(?:_impl|_config|<)", name)
        return "rocprim::" + (kind.group(1) if kind else "kernel")
    return name.split("(")[0][-60:]


def kernel_stats(d):
    rows = []
    with open(os.path.join(d, "kt", "kt_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            rows.append({"kernel": short(r["Name"]), "calls": int(r["Calls"]),
                         "total_us": float(r["TotalDurationNs"]) / 1e3,
                         "avg_us": float(r["AverageNs"]) / 1e3,
                         "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
                         "pct": float(r["Percentage"])})
    return rows


def kernel_resources(d):
    seen = {}
    with open(os.path.join(d, "kt", "kt_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if k not in seen:
                seen[k] = {"kernel": k, "vgpr": int(r["VGPR_Count"]),
                           "agpr": int(r["Accum_VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                           "lds_bytes": int(r["LDS_Block_Size"]),
                           "scratch_bytes": int(r["Scratch_Size"]),
                           "workgroup": int(r["Workgroup_Size_X"]), "grid": int(r["Grid_Size_X"])}
    return list(seen.values())


def pmc(d):
    agg = defaultdict(list)
    for sub in os.listdir(d):
        f = os.path.join(d, sub, "pmc_counter_collection.csv")
        if not sub.startswith("pmc_") or not os.path.exists(f):
            continue
        with open(f) as fh:
            for r in csv.DictReader(fh):
                agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    rnd = sys.argv[1]
    wls = sys.argv[2:] or ["tas", "gas", "deschedule"]
    os.makedirs(OUT, exist_ok=True)
    tpath = os.path.join(OUT, "traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for w in wls:
        d = os.path.join(ROOT, "gpurun_out", f"prof_{w}")
        rows = kernel_stats(d)
        with open(os.path.join(OUT, f"{rnd}_{w}_kernel_stats.csv"), "w", newline="") as f:
            wr = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            wr.writeheader()
            wr.writerows(rows)
        res = kernel_resources(d)
        with open(os.path.join(OUT, f"{rnd}_{w}_kernel_resources.csv"), "w", newline="") as f:
            wr = csv.DictWriter(f, fieldnames=list(res[0].keys()))
            wr.writeheader()
            wr.writerows(res)
        p = pmc(d)
        kernels = sorted({k for k, _ in p})
        counters = sorted({c for _, c in p})
        with open(os.path.join(OUT, f"{rnd}_{w}_pmc.csv"), "w", newline="") as f:
            wr = csv.writer(f)
            wr.writerow(["kernel"] + counters + ["hbm_bytes_per_launch"])
            for k in kernels:
                vals = [p.get((k, c), "") for c in counters]
                b = 1024 * (2 * p.get((k, "FETCH_SIZE"), 0) + p.get((k, "WRITE_SIZE"), 0))
                wr.writerow([k] + vals + [round(b)])

        def hbm(k):
            return 1024 * (2 * p.get((k, "FETCH_SIZE"), 0) + p.get((k, "WRITE_SIZE"), 0))
        if w == "tas":
            traffic["tas_path"] = round(sum(hbm(k) for k in TAS_PATH))
            traffic["tas_path_by_kernel"] = {k: round(hbm(k)) for k in TAS_PATH}
        elif w == "gas":
            # per step: gas_minfree_kernel runs once per snapshot change, not per fit
            calls = {r["kernel"]: r["calls"] for r in rows}
            per = max(calls.get("gas_rfit_single_kernel", 1), 1)
            wt = {k: min(calls.get(k, per) / per, 1.0) for k in GAS_PATH}
            traffic["gas_fit_kernel"] = round(sum(hbm(k) * wt[k] for k in GAS_PATH))
            traffic["gas_fit_by_kernel"] = {k: round(hbm(k)) for k in GAS_PATH}
            traffic["gas_fit_launches_per_step"] = {k: round(wt[k], 4) for k in GAS_PATH}
            # VALU wave-instructions per step (the fit kernels are issue-bound, not HBM-bound)
            if any(p.get((k, "SQ_INSTS_VALU")) for k in GAS_PATH):
                traffic["gas_fit_valu_per_step"] = round(
                    sum(p.get((k, "SQ_INSTS_VALU"), 0) * wt[k] for k in GAS_PATH))
                traffic["gas_fit_salu_per_step"] = round(
                    sum(p.get((k, "SQ_INSTS_SALU"), 0) * wt[k] for k in GAS_PATH))
                traffic["gas_fit_valu_by_kernel"] = {
                    k: round(p.get((k, "SQ_INSTS_VALU"), 0)) for k in GAS_PATH}
        elif w == "deschedule":
            # the sweep kernel (tas_violations_run_kernel since round 2), under the bench's key
            traffic["tas_violations_kernel"] = round(hbm("tas_violations_run_kernel") or
                                                     hbm("tas_violations_kernel"))
            traffic["label_plan_kernel"] = round(hbm("label_plan_kernel"))
        elif w == "c5":
            traffic["c5_by_kernel"] = {k: round(hbm(k)) for k in kernels}
        print(w, "->", [r["kernel"] + f" {r['avg_us']:.1f}us x{r['calls']}" for r in rows[:8]])
    traffic["_source"] = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, round {rnd}; "
                          "bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KB->B); "
                          "gas_fit_valu/salu_per_step: SQ_INSTS_VALU / SQ_INSTS_SALU pass")
    with open(tpath, "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
