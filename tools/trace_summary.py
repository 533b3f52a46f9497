"""Summarise a rocprofv3 --kernel-trace of `bench.py` (step workload): per pnp_step call the
compact kernel and the full / wide kernels' resume passes, split into the settle phase and the
timed steps.
usage: python tools/trace_summary.py <run_kernel_trace.csv> <timed_steps> [cmd-description]"""
import csv
import sys


def main():
    path, timed = sys.argv[1], int(sys.argv[2])
    desc = sys.argv[3] if len(sys.argv) > 3 else "bench.py"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        if "pnp_compact::step_kernel" in name:
            cur = [dur, 0.0, 0.0]
            calls.append(cur)
        elif "pnp_full::step_kernel" in name and cur is not None:
            cur[1] = dur
        elif "pnp_wide::step_kernel" in name and cur is not None:
            cur[2] = dur
            cur = None
    if len(calls) < timed:
        raise SystemExit(f"only {len(calls)} pnp_step calls in the trace")
    settle, tail = calls[:-timed], calls[-timed:]
    out = [f"rocprofv3 --kernel-trace of `{desc}` ({path.split('/')[-1]}), in launch order"]
    out.append(f"settle / warm-up phase ({len(settle)} pnp_step calls before the timed steps):")
    out += [f"  compact {c:8.3f} ms  full resume {r:8.3f} ms  wide resume {w:8.3f} ms" for c, r, w in settle]
    out.append(f"timed steps (last {timed} calls):")
    out += [f"  compact {c:8.3f} ms  full resume {r * 1e3:6.1f} us  wide resume {w * 1e3:6.1f} us" for c, r, w in tail]
    ca = sum(c for c, _, _ in tail) / timed
    ra = sum(r for _, r, _ in tail) / timed
    wa = sum(w for _, _, w in tail) / timed
    out.append(f"timed average: compact {ca:.3f} ms, full resume pass {ra * 1e3:.1f} us, wide resume pass "
               f"{wa * 1e3:.1f} us, sum {ca + ra + wa:.3f} ms")
    print("\n".join(out))


if __name__ == "__main__":
    main()
