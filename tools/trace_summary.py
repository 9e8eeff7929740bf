"""Summarise SVAE_TRACE_GEMM lines (stderr of one bench step with --warmup 1 --steps 1): per layer
shape, launches, average and total isolated time.   python tools/trace_summary.py trace.err [grep]"""
import collections
import re
import sys

lines = [l for l in open(sys.argv[1]) if l.startswith("GEMM")]
last = lines[len(lines) // 2:]  # the timed step
pat = sys.argv[2] if len(sys.argv) > 2 else None
d = collections.defaultdict(list)
for l in last:
    key = re.sub(r"\s+[\d.]+ us.*", "", l.strip())[5:]
    d[key].append((float(re.search(r"([\d.]+) us", l).group(1)), float(re.search(r"([\d.]+) TF/s", l).group(1))))
tot = sum(u for v in d.values() for u, _ in v)
print("total %.1f us over %d launches" % (tot, len(last)))
for k, v in sorted(d.items(), key=lambda kv: -sum(u for u, _ in kv[1])):
    if pat and not re.search(pat, k):
        continue
    print("%-92s x%2d avg %7.2f us tot %7.1f %6.1f TF/s" % (k, len(v), sum(u for u, _ in v) / len(v),
                                                         sum(u for u, _ in v), sum(t for _, t in v) / len(v)))
