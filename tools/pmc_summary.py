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

pmc_summary.json holds one entry per workload (its node count) under each
timed group of the library (the names bench.py's roofline uses): a group's
traffic per launch is the sum over the kernels its launch issues (GROUPS),
each launched once per group launch.  Earlier workloads' entries are kept.
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


# timed group (libnemohip's nemo_timings names) -> rocprof kernel base names issued inside it
GROUPS = {
    "k_build": ["k_build"],
    "k_csr": ["k_load_sel", "k_csr"],
    "k_csrb": ["k_cb_zero", "k_cb_hist", "k_cb_scan", "k_cb_part", "k_cb_bucket", "k_csrb_fin", "k_csrb_zero",
               "k_csrb_count", "k_csrb_scan", "k_csrb_scatter", "k_csrb_rows"],
    "k_topo": ["k_topo", "k_topo_deep"],
    "k_marksimp": ["k_marksimp"],
    "k_mark": ["k_mark", "k_mw_mark_z", "k_mw_mark_a", "k_mw_mark_b"],
    "k_simplify": ["k_simplify_flags", "k_mw_simplify_1", "k_mw_simplify_2", "k_mw_simplify_3", "k_mw_simplify_4"],
    "k_chains": ["k_chains", "k_chains_sel", "k_chains_list", "k_chains_big", "k_glob_prep", "k_chains_glob"],
    "k_proto": ["k_proto_lds", "k_proto_sel", "k_pg_init", "k_pg_link", "k_pg_a", "k_pg_b", "k_pg_c", "k_pg_sweep",
                "k_pg_d", "k_pg_gate"],
    "k_pull": ["k_pull_lds", "k_pull_sel", "k_pull", "k_mwp_count", "k_mwp_scan", "k_mwp_write", "k_scan64"],
    # the multi-entry kernels (k_dx.hip; k_zero's two small clears are not attributed) and the
    # one-workgroup-per-entry ones (option diff_legacy)
    "k_diff": ["k_dx_label", "k_dx_good", "k_dx_walks", "k_dx_lc", "k_dx_lp", "k_dx_emit", "k_dx_mask",
               "k_dprep_a", "k_dprep_scan", "k_dprep_b", "k_diff_lds", "k_diff", "k_diff_expand"],
}


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
    path = os.path.join(prof, "pmc_summary.json")
    try:
        summary = json.load(open(path))
        if "_rule" in summary and not summary.get("_per_workload"):
            summary = {}  # the round-2 layout (one workload): superseded
    except (OSError, ValueError):
        summary = {}
    for grp, members in GROUPS.items():
        parts = [base_hbm[m] for m in members if m in base_hbm]
        if not parts:
            continue
        hbm = sum(p[0] for p in parts)
        if grp == "k_diff" and bj["config"].get("diff_mode") == "per_run":
            grp = "k_diff_per_run"  # bench.py's roofline_diff (a run with --diff-mode per_run: every launch per-run)
        summary.setdefault(grp, {})[str(nodes)] = {
            "hbm_bytes_per_launch": round(hbm), "fetch_kib": round(sum(p[1] for p in parts), 1),
            "write_kib": round(sum(p[2] for p in parts), 1), "kernels": [m for m in members if m in base_hbm],
            "round": tag, "config": bj["config"].get("workload", "")[:40]}
    summary["_rule"] = ("2*FETCH_SIZE + WRITE_SIZE, KiB->bytes, per launch of the timed group (the sum over the "
                        "kernels it issues), keyed by the workload's node count")
    summary["_per_workload"] = True
    json.dump(summary, open(path, "w"), indent=1)
    open(os.path.join(prof, f"{tag}_pmc.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
