"""Summarise a tools/prof_bench.sh output directory into profiles/.

usage: python tools/pmc_summary.py gpurun_out/prof_<name> <round tag>

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `python3 bench.py`
  profiles/<tag>_bench.json         the bench line of the unprofiled run
  profiles/<tag>_pmc.md             per-kernel HBM bytes + SQ counters per launch
  profiles/pmc_summary.json         per-launch HBM traffic per kernel (bench.py's roofline.traffic)
HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE tallies 128-B read requests at 64 B (MI355X_MICROARCH.md, HBM
section), WRITE_SIZE is exact for wide stores.  Other widths are uncalibrated.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "", 1).replace("nemo::", "")


def per_kernel(pattern, counter=None):
    acc = defaultdict(lambda: defaultdict(list))
    for r in rows(pattern):
        if not r["Kernel_Name"].replace("void ", "", 1).startswith("nemo::"):
            continue
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    d, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1]
    bj = json.loads(bench)
    open(os.path.join(prof, f"{tag}_bench.json"), "w").write(bench + "\n")
    fetch = per_kernel(os.path.join(d, "pmc_fetch", "**", "*counter_collection.csv"))
    write = per_kernel(os.path.join(d, "pmc_write", "**", "*counter_collection.csv"))
    sq = per_kernel(os.path.join(d, "pmc_sq", "**", "*counter_collection.csv"))
    nodes = bj["config"]["nodes_total_rank0"]
    lines = [f"# {tag}: PMC per launch, bench.py workload ({nodes} nodes)", "",
             "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE correction); SQ cycles are quad-cycles.", "",
             "| kernel | launches | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM MB/launch | alg MB/launch | SQ_WAVES | "
             "WAIT_ANY % | WAIT_INST % | ACTIVE % | LDS insts | VALU insts |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    kern = bj.get("kernels", {})
    base_hbm = defaultdict(lambda: [0.0, 0.0, 0.0, 0])  # template tiers (k_chains<H, U>) add up per base kernel
    for k in sorted(fetch, key=lambda k: -sum(fetch[k]["FETCH_SIZE"])):
        f = fetch[k]["FETCH_SIZE"]
        w = write.get(k, {}).get("WRITE_SIZE", [0.0])
        n = len(f)
        fk, wk = sum(f) / n, sum(w) / max(1, len(w))
        hbm = (2 * fk + wk) * 1024
        s = sq.get(k, {})
        def m(c):
            v = s.get(c, [])
            return sum(v) / len(v) if v else 0.0
        cyc = m("SQ_WAVE_CYCLES") or 1.0
        alg = None
        if k in kern and bj["roofline"]["kernel"] == k:
            alg = bj["roofline"]["bytes_per_launch"]
        lines.append(f"| {k} | {n} | {fk:.0f} | {wk:.0f} | {hbm / 1e6:.1f} | {alg / 1e6 if alg else float('nan'):.1f} | "
                     f"{m('SQ_WAVES'):.0f} | {100 * m('SQ_WAIT_ANY') / cyc:.1f} | {100 * m('SQ_WAIT_INST_ANY') / cyc:.1f} | "
                     f"{100 * m('SQ_ACTIVE_INST_ANY') / cyc:.1f} | {m('SQ_INSTS_LDS'):.0f} | {m('SQ_INSTS_VALU'):.0f} |")
        b = base_hbm[k.split("<")[0]]
        b[0] += hbm
        b[1] += fk
        b[2] += wk
        b[3] = max(b[3], n)
    summary = {k: {"workload_nodes": nodes, "hbm_bytes_per_launch": round(hbm), "fetch_kib": round(fk, 1),
                   "write_kib": round(wk, 1), "launches": n, "round": tag}
               for k, (hbm, fk, wk, n) in sorted(base_hbm.items())}
    summary["_rule"] = "2*FETCH_SIZE + WRITE_SIZE, KiB->bytes (summed over template tiers)"
    json.dump(summary, open(os.path.join(prof, "pmc_summary.json"), "w"), indent=1)
    open(os.path.join(prof, f"{tag}_pmc.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
