"""Condense rocprofv3 CSV output into the small files committed under profiles/.

  python tools/rocprof_summary.py stats <kernel_stats.csv> [--top 25]
      -> markdown table: kernel (template arguments elided), calls, avg/min/max us, total ms, %
  python tools/rocprof_summary.py trace <kernel_trace.csv> --match gae_kernel
      -> JSON per (kernel, grid): dispatch count and avg/median/min/max duration
  python tools/rocprof_summary.py timeline <kernel_trace.csv> --match flatten_wide [--upto X]
      -> busy / idle-gap table per kernel from the last matching dispatch on, and the sequence
  python tools/rocprof_summary.py pmc <counter_collection.csv> [<more.csv> ...] --match gae_kernel
      -> JSON per (kernel, grid): dispatches, mean counter values per dispatch; FETCH_SIZE is
         also reported doubled (gfx950: FETCH_SIZE counts 1/2 of a wide streaming read,
         MI355X_MICROARCH.md HBM section), the figure bench.py's roofline.traffic uses.
"""
import argparse
import csv
import json
import sys
from collections import defaultdict


def short(name, width=110):
    s = name
    if s.endswith(")"):                        # drop the trailing parameter list
        depth = 0
        for i in range(len(s) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(s[i], 0)
            if depth == 0:
                s = s[:i]
                break
    depth, out = 0, []
    for ch in s:                               # elide nested template arguments
        if ch == "<":
            depth += 1
            if depth == 1:
                out.append("<")
            continue
        if ch == ">":
            depth -= 1
            if depth == 0:
                out.append(">")
            continue
        if depth <= 1:
            out.append(ch)
    s = "".join(out)
    return s if len(s) <= width else s[:width - 3] + "..."


def stats(path, top):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print("| kernel | calls | avg us | min us | max us | total ms | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in rows[:top]:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
              f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
              f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    rest = rows[top:]
    if rest:
        print(f"| ({len(rest)} more kernels) | {sum(int(r['Calls']) for r in rest)} | | | | "
              f"{sum(float(r['TotalDurationNs']) for r in rest) / 1e6:.3f} | "
              f"{sum(float(r['Percentage']) for r in rest):.2f} |")


def pmc(paths, match, n=0):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            if match and match not in r["Kernel_Name"]:
                continue
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for (k, grid), ctrs in sorted(acc.items()):
        e = {"kernel": k, "grid_size": grid}
        for c, v in ctrs.items():
            e[c] = {"dispatches": len(v), "mean": sum(v) / len(v)}
            if n:
                e["n"] = n
            if c == "FETCH_SIZE":   # KiB; x2 on gfx950
                e["read_bytes_corrected"] = 2 * 1024 * sum(v) / len(v)
            if c == "WRITE_SIZE":
                e["write_bytes"] = 1024 * sum(v) / len(v)
        out.append(e)
    print(json.dumps(out[0] if n and len(out) == 1 else out, indent=1))


def trace(path, match, last=0):
    """Durations of the matching kernel's dispatches, grouped by grid size; last > 0 keeps only
    the last `last` dispatches of each group in time order (e.g. bench.py's timed steps after
    its warm-up launch)."""
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            acc[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(
                (int(r["Start_Timestamp"]),
                 (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = []
    for (k, grid), ev in sorted(acc.items()):
        ev.sort()
        n_all = len(ev)
        if last > 0:
            ev = ev[-last:]
        us = sorted(d for _, d in ev)
        out.append({"kernel": k, "grid_size": grid, "dispatches": n_all,
                    "averaged_over": ("all" if last <= 0 or last >= n_all
                                      else f"last {len(us)} in time order"),
                    "avg_us": round(sum(us) / len(us), 2), "median_us": us[len(us) // 2],
                    "min_us": us[0], "max_us": us[-1]})
    print(json.dumps(out, indent=1))


def timeline(path, match, upto=""):
    """The GPU timeline from the last dispatch matching `match` (e.g. the rollout's flatten, right
    before learn()) to the end or to the next `upto` dispatch: per kernel, dispatches, busy time
    and the idle gap before its dispatches (host launch / sync time), then the run-length-
    compressed sequence."""
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"], 70))
                for r in csv.DictReader(open(path)))
    i0 = max(i for i, e in enumerate(ev) if match in e[2])
    ev = ev[i0:]
    if upto:
        ends = [i for i, e in enumerate(ev) if i > 0 and upto in e[2]]
        if ends:
            ev = ev[:ends[0]]
    per = defaultdict(lambda: [0, 0.0, 0.0])
    seq = []
    prev_end = ev[0][0]
    for st, en, k in ev:
        gap = max(0.0, (st - prev_end) / 1e3)
        prev_end = max(prev_end, en)
        p_ = per[k]
        p_[0] += 1
        p_[1] += (en - st) / 1e3
        p_[2] += gap
        if seq and seq[-1][0] == k:
            seq[-1][1] += 1
            seq[-1][2] += (en - st) / 1e3
            seq[-1][3] += gap
        else:
            seq.append([k, 1, (en - st) / 1e3, gap])
    win = (ev[-1][1] - ev[0][0]) / 1e3
    busy = sum(v[1] for v in per.values())
    print(f"window {win / 1e3:.3f} ms, busy {busy / 1e3:.3f} ms, idle {(win - busy) / 1e3:.3f} ms, "
          f"{len(ev)} dispatches")
    print("| kernel | n | busy us | gap before us |\n|---|---:|---:|---:|")
    for k, (n, b, g) in sorted(per.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
        print(f"| `{k}` | {n} | {b:.1f} | {g:.1f} |")
    print("\nsequence (kernel x n: busy us, gap us):")
    for k, n, b, g in seq[:160]:
        print(f"  {k} x{n}: {b:.1f}, gap {g:.1f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["stats", "pmc", "trace", "timeline"])
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default="")
    ap.add_argument("--n", type=int, default=0, help="pmc: transitions per launch (recorded)")
    ap.add_argument("--upto", default="", help="timeline: stop at the next matching dispatch")
    ap.add_argument("--last", type=int, default=0, help="trace: average the last N dispatches")
    a = ap.parse_args()
    if a.mode == "stats":
        stats(a.paths[0], a.top)
    elif a.mode == "pmc":
        pmc(a.paths, a.match, a.n)
    elif a.mode == "timeline":
        timeline(a.paths[0], a.match, a.upto)
    else:
        trace(a.paths[0], a.match, a.last)
