"""Per-dispatch averages of rocprofv3 --pmc CSV counter collections for one kernel.
usage: python tools/sq_summary.py <pass_dir> [<pass_dir> ...] <kernel-name-substring> [--json out.json --waves-per-simd N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    argv = sys.argv[1:]
    jpath, wps = None, 2
    if "--json" in argv:
        i = argv.index("--json")
        jpath = argv[i + 1]
        del argv[i:i + 2]
    if "--waves-per-simd" in argv:
        i = argv.index("--waves-per-simd")
        wps = int(argv[i + 1])
        del argv[i:i + 2]
    dirs, kname = argv[:-1], argv[-1]
    tot = defaultdict(float)
    nd = defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kname not in r["Kernel_Name"]:
                    continue
                c = r["Counter_Name"]
                tot[c] += float(r["Counter_Value"])
                nd[c].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    if not tot:
        raise SystemExit(f"no rows for {kname}")
    per = {c: tot[c] / max(1, len(nd[c])) for c in tot}
    print(f"{kname}: per-dispatch averages")
    for c in sorted(per):
        print(f"  {c:24s} {per[c]:16.0f}  ({len(nd[c])} dispatches)")
    w = per.get("SQ_WAVES", 0)
    if w:
        print("per wave:")
        for c in sorted(per):
            if c != "SQ_WAVES":
                print(f"  {c:24s} {per[c] / w:14.1f}")
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if c in per:
                print(f"  {c} / SQ_WAVE_CYCLES = {per[c] / wc:.3f}")
        if "SQ_INSTS_VALU" in per:
            print(f"  VALU pipe utilisation (2 cycles per VALU instruction, SQ_WAVE_CYCLES in quad-cycles, "
                  f"{wps} waves per SIMD) = {min(1.0, wps * 2.0 * per['SQ_INSTS_VALU'] / (4.0 * wc)):.3f}")
    if jpath and wc and "SQ_ACTIVE_INST_VALU" in per:
        import json
        rec = {"kernel": kname, "waves_per_simd": wps,
               "wave_frac": {c: per[c] / wc for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                                                     "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY") if c in per},
               "insts_per_wave": {c: per[c] / w for c in per if c.startswith("SQ_INSTS_") and w},
               # the SIMD's vector ALU: each resident wave keeps it busy its own ACTIVE_INST_VALU share
               "valu_issue_frac": min(1.0, wps * per["SQ_ACTIVE_INST_VALU"] / wc),
               # VALU pipe utilisation from instruction counts: a wave64 VALU instruction occupies the
               # SIMD's pipe 2 cycles (MI355X_MICROARCH.md, hardware model) and SQ_WAVE_CYCLES counts
               # quad-cycles (its PMC-units row), so a wave keeps the pipe busy 2 x SQ_INSTS_VALU of its
               # 4 x SQ_WAVE_CYCLES, times the resident waves per SIMD
               "valu_pipe_util": (min(1.0, wps * 2.0 * per["SQ_INSTS_VALU"] / (4.0 * wc)) if "SQ_INSTS_VALU" in per else None),
               "source": "rocprofv3 --pmc SQ_* (two passes of 8 SQ counters), tools/gpu.sh sq"}
        json.dump(rec, open(jpath, "w"), indent=1)


if __name__ == "__main__":
    main()
