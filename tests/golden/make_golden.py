"""Regenerate tests/golden/*.npz from the CPU oracle (run from the repo root:
python tests/golden/make_golden.py).  The oracle is a restatement of the
reference's algorithm (oracle/gar_oracle.c); see golden_cases.py."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.dirname(HERE)]

import golden_cases  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    O.build()
    for case in golden_cases.CASES:
        outs = golden_cases.run_oracle(O, case)
        golden_cases.save(case, outs)
        print(case["name"], [len(o) for o in outs])
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (CPU oracle oracle/gar_oracle.c)",
                   "cases": golden_cases.CASES}, f, indent=1)


if __name__ == "__main__":
    main()
