"""HBM traffic per launch of one kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

usage: python tools/pmc_traffic.py KERNEL LAST TRACE_DIR FETCH_DIR WRITE_DIR > profiles/r01/<k>_pmc.json

FETCH_SIZE and WRITE_SIZE come from separate --pmc runs of the same command (one TCC budget each),
in KB per dispatch.  On gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so it is
doubled; WRITE_SIZE is taken as is.  LAST = the number of trailing launches to average (the timed
region); the kernel-trace directory gives the same launches' mean duration for cross-checking
the HIP-event time bench.py reports.
"""
import csv
import glob
import json
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, pat))[0]
    out = list(csv.DictReader(open(f)))
    key = "Start_Timestamp" if "Start_Timestamp" in out[0] else "Dispatch_Id"
    out.sort(key=lambda r: int(r[key]))
    return out


def short(n):
    return n.split("(")[0].replace("tr::", "")


def main(kern, last, tdir, fdir, wdir):
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
           for r in rows(tdir, "*kernel_trace.csv") if short(r["Kernel_Name"]) == kern][-last:]
    per = {}
    for d, ctr in ((fdir, "FETCH_SIZE"), (wdir, "WRITE_SIZE")):
        v = [float(r["Counter_Value"]) for r in rows(d, "*counter_collection.csv")
             if short(r["Kernel_Name"]) == kern and r["Counter_Name"] == ctr][-last:]
        per[ctr] = sum(v) / len(v) if v else None
    fetch = None if per["FETCH_SIZE"] is None else 2 * per["FETCH_SIZE"] * 1024
    write = None if per["WRITE_SIZE"] is None else per["WRITE_SIZE"] * 1024
    out = {"kernel": kern, "launches": len(dur), "mean_us": sum(dur) / len(dur) if dur else None,
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": None if fetch is None or write is None else fetch + write,
           "correction": "FETCH_SIZE x2 (gfx950 wide reads), KB x 1024"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), *sys.argv[3:6])
