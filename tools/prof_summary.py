#!/usr/bin/env python3
"""rocprofv3 kernel_stats.csv -> markdown table (profiles/<round>/*_summary.md)."""
import csv
import sys


def main():
    src, title = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(src)))
    print(f"# {title}\n")
    print("| kernel | calls | avg ms | total % |")
    print("|---|---|---|---|")
    for r in rows:
        print(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
