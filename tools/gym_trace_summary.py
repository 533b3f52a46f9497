"""Per gym step, the env-step passes from a rocprofv3 --kernel-trace of bench.py's gym leg: each
pass's tier, start offset and duration (ms) and the step's span.  A step ends with its
route_commit_kernel (env_dev.h, with a tier buffer) or, without one, at the next compact pass.
usage: python tools/gym_trace_summary.py <run_kernel_trace.csv> [last_n]"""
import csv
import sys


def tier_of(name):
    for key, tag in (("pnp_compact_gym::", "compact"), ("pnp_full::", "full"), ("pnp_wide::", "wide")):
        if key in name:
            return tag
    return "?"


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    commit = any("route_commit_kernel" in r["Kernel_Name"] for r in rows)
    for r in rows:
        name = r["Kernel_Name"]
        if "route_commit_kernel" in name:
            if cur:
                steps.append(cur)
            cur = []
        elif "env_step_kernel" in name or "env_step_wide_kernel" in name:
            if not commit and "pnp_compact_gym::" in name and cur:
                steps.append(cur)
                cur = []
            cur.append((tier_of(name), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if cur and not commit:
        steps.append(cur)
    print(f"{len(steps)} gym steps in {path.split('/')[-1]}; last {last} (pass: start offset + duration, ms):")
    spans = []
    for st in steps[-last:]:
        t0 = min(s for _, s, _ in st)
        span = (max(e for _, _, e in st) - t0) * 1e-6
        spans.append(span)
        print(f"  span {span:7.2f}  " + "  ".join(f"{t} +{(s - t0) * 1e-6:.1f} {(e - s) * 1e-6:.1f}" for t, s, e in st))
    if spans:
        print(f"  mean span {sum(spans) / len(spans):.2f} ms")


if __name__ == "__main__":
    main()
