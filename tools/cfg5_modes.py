#!/usr/bin/env python3
"""cfg5 per-kind kernel ms per launch (decimator on bg_rt_kernel, composite on bg_rb_kernel) for one
GAR_BG_DBG mode: python3 tools/cfg5_modes.py (env GAR_BG_DBG, GAR_LIB_PATH as usual)."""
import json
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = subprocess.run([sys.executable, os.path.join(R, "bench.py"), "--workload", "cfg5", "--steps", "4", "--warmup", "2",
                    "--no-cpu-baseline", "--no-pmc", "--no-streaming", "--check-seconds", "0", "--secondary", "none"],
                   capture_output=True, text=True, timeout=300)
if p.returncode:
    sys.stderr.write(p.stderr[-3000:])
    sys.exit(p.returncode)
d = json.loads(p.stdout.strip().splitlines()[-1])
r = d["roofline"]
per = {k: round(v / max(r["launches_per_step_by_kind"][k], 1) * 1e3, 2) for k, v in r["kernel_ms_by_kind"].items()}
print("GAR_BG_DBG", os.environ.get("GAR_BG_DBG", "0"), "value", d["value"], "ms_per_step", d["ms_per_step"], "us per launch", per)
