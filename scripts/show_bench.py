"""Print the headline fields of a bench.py JSON line (the last line of the given file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["kernels_ms"])
c5 = d.get("extra_configs", {}).get("config5", {})
print(c5.get("one_channel"), c5.get("channels_1024"))
