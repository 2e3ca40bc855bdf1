"""Molly-format outputs of the reference's six case studies,
produced by nemo_amd.molly from /root/reference/case-studies/*.ded with the
flags quoted in each program, plus expected.json from the literal restatement
(oracle/cypher_literal.py + oracle/host_literal.py), like make_fixtures.py.

Only the generated data is committed (tests/golden/cs_<name>/); the programs
themselves stay in the reference.  Run here (the reference is not on the GPU
box):  python tests/golden/make_case_studies.py
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from nemo_amd.molly import explore, parse, write_output  # noqa: E402
from tests.golden.make_fixtures import expected  # noqa: E402

CASES = "/root/reference/case-studies"
MAX_RUNS = 24


def main():
    for fn in sorted(os.listdir(CASES)):
        if not fn.endswith(".ded"):
            continue
        name = "cs_" + fn[:-4].replace("-", "_").lower()
        with open(os.path.join(CASES, fn)) as fh:
            prog = parse(fh.read())
        o = prog.options
        runs = explore(prog, int(o["EOT"]), int(o["EFF"]), int(o.get("crashes", 0)), o["nodes"].split(","),
                       max_runs=MAX_RUNS)
        d = os.path.join(HERE, name)
        shutil.rmtree(d, ignore_errors=True)
        write_output(runs, d, indent=None)
        meta = json.load(open(os.path.join(d, "runs.json")))
        spec = []
        for i, r in enumerate(meta):
            pre = json.load(open(os.path.join(d, f"run_{i}_pre_provenance.json")))
            post = json.load(open(os.path.join(d, f"run_{i}_post_provenance.json")))
            spec.append((r["iteration"], r["status"], pre, post))
        exp = expected(spec, digests=True)
        exp["source"] = {"program": f"case-studies/{fn}", "eot": int(o["EOT"]), "eff": int(o["EFF"]),
                         "crashes": int(o.get("crashes", 0)), "nodes": o["nodes"], "max_runs": MAX_RUNS}
        with open(os.path.join(d, "expected.json"), "w") as fh:
            json.dump(exp, fh, sort_keys=True, separators=(",", ":"))
        print(f"wrote {name}: {len(runs)} runs, {sum(not r.success for r in runs)} failed")


if __name__ == "__main__":
    main()
