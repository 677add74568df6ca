"""One row per bench.py JSON file: value, step (in flight and one at a time), scan-kernel
time by the bench's HIP events and its roofline fraction.  Used to condense same-box A/B
runs (profiles/r06_run*.sh) into profiles/r06_ab/*.txt.
Usage: ab_table.py <title> <file.json> [...]   (the last line of each file is the JSON)"""
import json
import os
import sys


def main(title, files):
    print(f"# {title}")
    print(f"{'run':<28} {'queries/s':>11} {'step ms':>8} {'serial ms':>9} {'scan us':>8} {'frac':>6} {'repairs':>7}")
    for f in files:
        try:
            j = json.loads(open(f).read().strip().splitlines()[-1])
        except Exception as e:  # a failed run: say so
            print(f"{os.path.basename(f):<28} unreadable ({e})")
            continue
        r = j.get("roofline", {})
        print(f"{os.path.basename(f):<28} {j['value']:>11.0f} {j['ms_per_step']:>8.4f} "
              f"{j.get('ms_per_step_serial') or float('nan'):>9.4f} {1e3 * r.get('avg_launch_ms', float('nan')):>8.1f} "
              f"{r.get('frac', float('nan')):>6.3f} {str(j.get('repairs')):>7}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
