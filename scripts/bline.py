"""Print the key fields of bench.py JSON lines: python scripts/bline.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    for l in open(f):
        l = l.strip()
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        st = d.get("stages_ms", {})
        print(f, d["value"], "ms/step", d["ms_per_step"], "lat", d.get("latency_ms_per_encode"),
              {k: v for k, v in st.items() if k.endswith("_ms")}, "verified", (d.get("verified") or {}).get("ok"))
