#!/usr/bin/env python3
"""Summarise an interleaved A/B log written by scripts/gpu_cnn_env_ab.sh ("round R VARIANT {json}")."""
import collections
import json
import re
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"round (\d+) (\S+) (\{.*)", line)
    if m:
        j = json.loads(m.group(3))
        d[m.group(2)].append((j["value"], j["ms_per_step"]))
base = None
for k, v in d.items():
    mean = sum(x for x, _ in v) / len(v)
    base = base or mean
    print(f"{k:32s} {' '.join(f'{x:.1f}' for x, _ in v)}  mean {mean:.1f}  ({100 * (mean / base - 1):+.2f} %)")
