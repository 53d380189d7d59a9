"""Graph-mode timeline of a rocprofv3 --kernel-trace CSV: over the last `frac` of the run (the timed
steps), per kernel family the summed time and count, the union of busy intervals, idle gaps and
the time two or more kernels overlap.

    python tools/graph_gaps.py gpurun_out/gtrace/run_kernel_trace.csv.gz [frac=0.4] [iters]
"""
import csv, gzip, re, sys
from collections import defaultdict

def load(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        rows = list(csv.DictReader(f))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ev.sort()
    return ev

def family(name):
    n = name.replace("aa::(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*$", "", n)
    return n[:70]

def main():
    path = sys.argv[1]
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.4   # < 1: fraction of the run; >= 1: last `frac` us
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    ev = load(path)
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    cut = t1 - (frac * (t1 - t0) if frac < 1 else frac * 1e3)
    ev = [e for e in ev if e[0] >= cut]
    w0, w1 = ev[0][0], max(e[1] for e in ev)
    fam = defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        f = family(n); fam[f][0] += e - s; fam[f][1] += 1
    # union / overlap
    pts = sorted([(s, 1) for s, e, n in ev] + [(e, -1) for s, e, n in ev])
    busy = over = 0; depth = 0; last = pts[0][0]; gaps = []
    for t, d in pts:
        if depth >= 1: busy += t - last
        if depth >= 2: over += t - last
        if depth == 0 and t > last: gaps.append(t - last)
        depth += d; last = t
    wall = w1 - w0
    k = iters or 1
    print(f"window {wall/1e3:.1f} us, {len(ev)} kernels; busy {busy/1e3:.1f} us, idle {(wall-busy)/1e3:.1f} us, "
          f">=2 kernels {over/1e3:.1f} us" + (f"; per iteration ({iters}): wall {wall/1e3/k:.1f} us" if iters else ""))
    gaps.sort()
    if gaps:
        print(f"gaps: n {len(gaps)}, sum {sum(gaps)/1e3:.1f} us, median {gaps[len(gaps)//2]/1e3:.2f} us, "
              f">5us {sum(g for g in gaps if g > 5000)/1e3:.1f} us")
    for f, (t, c) in sorted(fam.items(), key=lambda x: -x[1][0])[:40]:
        print(f"{t/1e3/k:10.1f} us {c/k:8.2f} x  {f}")

if __name__ == "__main__":
    main()
