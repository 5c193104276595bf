"""Summarise QDC_RQ_STATS=1 stderr of a bench run: per call direction (the lines before
"forward plan+build" belong to that forward call, before "backward plan+build" to that
backward), the register-resident passes, their stages and ops (stages + relayouts + returns to
L0) and the tile sizes; the last call of each direction is reported."""
import re
import sys
from collections import Counter


def main(path):
    calls = {"forward": [], "backward": []}
    cur = []
    for line in open(path):
        m = re.match(r"rq pass: (\d+) stages, (\d+) ops \(T=(\d+) lc=(\d+)\)", line)
        if m:
            cur.append(tuple(int(x) for x in m.groups()))
            continue
        m = re.match(r"(forward|backward) plan\+build", line)
        if m:
            calls[m.group(1)].append(cur)
            cur = []
    for d, cs in calls.items():
        if not cs:
            continue
        ps = cs[-1]
        st = sum(p[0] for p in ps)
        ops = sum(p[1] for p in ps)
        print(f"{d}: {len(ps)} rq passes, {st} stages, {ops} ops ({ops - st} relayout/return ops, "
              f"{(ops - st) / max(len(ps), 1):.2f} per pass, {st / max(len(ps), 1):.2f} stages per pass), "
              f"tiles {dict(Counter(p[2] for p in ps))}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        main(p)
