"""python -m nemo_amd.molly PROGRAM.ded OUT_DIR [--nodes a,b] [--EOT n] [--EFF n] [--crashes n] [--max-runs n]

Flags default to the Molly command line quoted in the program's comments
(case-studies/*.ded:2)."""
import argparse
import sys

from .dedalus import parse
from .ldfi import explore, write_output


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m nemo_amd.molly")
    ap.add_argument("program")
    ap.add_argument("out_dir")
    ap.add_argument("--nodes")
    ap.add_argument("--EOT", type=int)
    ap.add_argument("--EFF", type=int)
    ap.add_argument("--crashes", type=int)
    ap.add_argument("--max-runs", type=int, default=32)
    a = ap.parse_args(argv)
    with open(a.program) as fh:
        prog = parse(fh.read())
    o = prog.options
    nodes = (a.nodes or o.get("nodes", "")).split(",")
    eot = a.EOT or int(o.get("EOT", 6))
    eff = a.EFF if a.EFF is not None else int(o.get("EFF", 4))
    crashes = a.crashes if a.crashes is not None else int(o.get("crashes", 0))
    runs = explore(prog, eot, eff, crashes, [n for n in nodes if n], max_runs=a.max_runs)
    write_output(runs, a.out_dir)
    n_fail = sum(not r.success for r in runs)
    print(f"{len(runs)} runs ({n_fail} failed) -> {a.out_dir}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
