"""Print tools/ab_libs.sh results: per (cfg, mode, lib) the event times of each round."""
import collections
import json
import sys

d = collections.defaultdict(list)
for ln in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_libs.txt"):
    if ln.startswith("{"):
        x = json.loads(ln)
        d[(x["cfg"], x["mode"], x.get("lib", "prod"))].append(x["event_us_per_call"])
for k in sorted(d):
    print(*k, d[k])
