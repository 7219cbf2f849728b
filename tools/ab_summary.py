"""Summarise tools/ab_seeds.sh / ab_bench.sh output lines ("tag rep value ms sha"): per variant the
mean ratio to `base` paired by seed / repetition, and whether its end states equal base's."""
import collections
import sys

rows = [ln.split() for ln in open(sys.argv[1]) if ln.strip() and len(ln.split()) == 5]
by = collections.defaultdict(dict)
for tag, rep, val, ms, sha in rows:
    by[tag][rep] = (float(val), sha)
base = by.get("base", {})
for tag, d in sorted(by.items()):
    common = [r for r in d if r in base]
    ratios = [d[r][0] / base[r][0] for r in common]
    same = all(d[r][1] == base[r][1] for r in common)
    mean = sum(v for v, _ in d.values()) / len(d)
    print(f"{tag:12s} mean {mean / 1e6:7.3f} M  ratio vs base {sum(ratios) / max(len(ratios), 1):.4f} "
          f"(n={len(ratios)}, min {min(ratios):.4f}, max {max(ratios):.4f}) {'bitwise-equal' if same else 'different states'}")
