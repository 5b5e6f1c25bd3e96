"""Per-launch durations of the bench's TIMED window from a rocprofv3 kernel trace (--kernel-trace, csv).

A kernel launched once per step has, in the trace of a `bench.py` command, the step ordinals as its dispatch indices:
the bench line's config.timed_steps = [a, b) selects the timed steps' dispatches.  For each probed launch (the
selectors of tools/pmc_summary.py) this prints the average over dispatches [a, b) and over all dispatches, as a
kernel-stats CSV (Name, Calls, AverageNs, WindowCalls, WindowAverageNs).

    python tools/rocprof_window.py <dir with *kernel_trace.csv> <bench json line file> > window_kernel_stats.csv"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import KERNELS, match  # noqa: E402


def main(d, bench):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    line = [x for x in open(bench).read().splitlines() if x.startswith("{")][-1]
    a, b = json.loads(line)["config"]["timed_steps"]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    w = csv.writer(sys.stdout)
    w.writerow(["Probe", "Name", "Calls", "AverageNs", "WindowFirst", "WindowCalls", "WindowAverageNs"])
    for probe, sel in KERNELS.items():
        if not probe.startswith("tgn_"):
            continue
        names = {r["Kernel_Name"] for r in rows if match(r["Kernel_Name"], sel)}
        for n in sorted(names):
            dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"] == n]
            win = dur[a:b]
            if not win:
                continue
            w.writerow([probe, n[:200], len(dur), round(sum(dur) / len(dur), 1), a, len(win),
                        round(sum(win) / len(win), 1)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
