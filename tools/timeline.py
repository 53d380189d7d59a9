"""Per-iteration timeline of a C4 kernel trace (graph mode): the last 100 k_aa_mix launches mark
iterations; between consecutive ones, GPU busy time (union of kernel intervals) vs wall, and the
kernels by name with their count and time -- gated launches (reject branch not taken) show up as
many short dispatches.

    python tools/timeline.py run_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def short(n):
    m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r)
        for r in csv.DictReader(open(sys.argv[1]))]
rows.sort()
marks = [i for i, r in enumerate(rows) if r[2].startswith("k_aa_mix")]
marks = marks[-101:]
busy = wall = 0
per = collections.defaultdict(lambda: [0, 0.0, 0])
for a, b in zip(marks[:-1], marks[1:]):
    seg = rows[a + 1:b + 1]
    t0, t1 = rows[a][1], rows[b][1]
    wall += t1 - t0
    cur_s = cur_e = None
    for s, e, n, _ in seg:
        per[n][0] += 1
        per[n][1] += (e - s) / 1e3
        if e - s < 4000:
            per[n][2] += 1
        s = max(s, t0)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
it = len(marks) - 1
print(f"iterations {it}: wall {wall / it / 1e3:.1f} us/iter, busy {busy / it / 1e3:.1f} us/iter, "
      f"idle {(wall - busy) / it / 1e3:.1f} us/iter, launches {sum(v[0] for v in per.values()) / it:.1f}/iter")
for n, (c, t, sh) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    print(f"  {n[:60]:60s} {c / it:6.2f}/iter {t / it:9.2f} us/iter  short(<4us) {sh / it:5.2f}/iter")
