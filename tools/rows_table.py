"""Render tools/rows_bench.py output (a JSON list of rows) as the DESIGN.md §6a table.

Usage: python tools/rows_table.py profiles/r02_rows.json
"""
import json
import sys


def fmt_roof(r):
    rf = r.get("roofline")
    if not rf:
        return "—"
    return f"{rf['achieved']:.2f} {rf['unit']} = {rf['frac']:.3f} of {rf['bound']}"


def main():
    rows = json.load(open(sys.argv[1]))
    print("| Row | Workload | Msamples/s | µs/call | Roofline | CPU 1-core Msamples/s | × CPU |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        cpu = r.get("cpu_baseline") or {}
        print(f"| {r['row']} | {r['workload']} | {r['value']:.1f} | {r['ms_per_call'] * 1e3:.1f} | {fmt_roof(r)} | "
              f"{cpu.get('value', '—')} | {r.get('speedup_vs_cpu', '—')} |")


if __name__ == "__main__":
    main()
