"""Busy / idle analysis of a rocprofv3 kernel trace: union of kernel intervals over the last N
steps (a step = the span between consecutive adamw_flat_kernel launches), largest idle gaps and
the kernels that follow them.  Usage: python scripts/gap_analysis.py run_kernel_trace.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
marks = [s for s, e, n, _ in ev if n.startswith("adamw_flat")]
marks = marks[::2] if len(marks) > 2 * nsteps else marks  # two AdamW launches per step
lo, hi = marks[-nsteps - 1], marks[-1]
sel = [x for x in ev if x[0] >= lo and x[0] < hi]
busy, cur_s, cur_e, gaps = 0, None, None, []
for s, e, n, st in sel:
    if cur_e is None:
        cur_s, cur_e = s, e
        continue
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, n, st))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
wall = hi - lo
print(f"{nsteps} steps: wall {wall / 1e6 / nsteps:.2f} ms/step, GPU busy {busy / 1e6 / nsteps:.2f} ms/step "
      f"({100 * busy / wall:.1f} %), idle {(wall - busy) / 1e6 / nsteps:.2f} ms/step in {len(gaps)} gaps")
gaps.sort(reverse=True)
for g, n, st in gaps[:15]:
    print(f"  {g / 1e3:8.1f} us before {n[:70]} (stream {st})")
