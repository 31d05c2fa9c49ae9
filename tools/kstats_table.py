#!/usr/bin/env python3
"""Compact table of a rocprofv3 ``*_kernel_stats.csv``: kernel, calls, avg us,
total %.  Usage: python tools/kstats_table.py <kernel_stats.csv> [--top 12]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    rows = list(csv.DictReader(open(path)))
    for r in rows[:top]:
        name = r.get("Name", "")
        m = re.search(r"(k_[A-Za-z0-9_]+(?:<[^>]*>)?)", name)
        short = m.group(1) if m else name[:50]
        avg = float(r.get("AverageNs", 0)) / 1e3
        print(f"{short:40s} calls {int(r.get('Calls', 0)):6d}  avg {avg:8.2f} us  {float(r.get('Percentage', 0)):6.2f} %")


if __name__ == "__main__":
    main()
