"""Tabulate tools/band_sweep.py JSON lines: us_per_rep per shape x fuse, per world."""
import json
import sys
from collections import defaultdict

rows = [json.loads(l) for f in sys.argv[1:] for l in open(f) if l.startswith("{")]
g = defaultdict(dict)
for r in rows:
    g[(r["world"], r["ch"])][(r["fuse"], r["shape"])] = r["us_per_rep"]
for k, d in g.items():
    fuses = sorted({f for f, _ in d})
    shapes = []
    for _, s in d:
        if s not in shapes:
            shapes.append(s)
    print(f"world={k[0]} ch={k[1]}")
    print("shape     " + "".join(f"{f:>8}" for f in fuses))
    for s in shapes:
        print(f"{s:9} " + "".join(f"{(d.get((f, s)) or float('nan')):8.3f}" for f in fuses))
