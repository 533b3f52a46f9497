"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes for one
kernel, corrected as MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE reads half the bytes of
a wide coalesced stream: doubled; WRITE_SIZE taken as is; both in KiB -> bytes).
usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <batch> <out.json> [last_n]
(last_n: average only the last n dispatches, i.e. the timed steps after bench.py's settle and
warm-up launches)"""
import csv
import glob
import json
import sys


def per_dispatch(d, counter, ksub):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if ksub in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append((int(row.get("Dispatch_Id", len(vals))), float(row["Counter_Value"])))
    return [v for _, v in sorted(vals)]


def main():
    fd, wd, ksub, batch, out = sys.argv[1:6]
    last = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    f = per_dispatch(fd, "FETCH_SIZE", ksub)[-last:]
    w = per_dispatch(wd, "WRITE_SIZE", ksub)[-last:]
    if not f or not w:
        raise SystemExit(f"no dispatches of {ksub!r} found (fetch {len(f)}, write {len(w)})")
    fetch = sum(f) / len(f) * 1024 * 2     # KiB -> B, x2 gfx950 FETCH_SIZE correction
    write = sum(w) / len(w) * 1024
    rec = {"kernel": ksub, "batch": int(batch), "dispatches": [len(f), len(w)],
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM section)"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
