#!/usr/bin/env python3
"""Turn rocprofv3 --pmc counter_collection.csv files into the compact summary
committed under profiles/*_pmc_*.csv (the format bench.py:pmc_traffic reads).

usage: tools/pmc_csv.py OUT.csv "CONFIG" "COMMAND" FETCH_DIR WRITE_DIR [KERNEL_SUBSTR]

CONFIG is the "workload=encode k=10 p=4 len=1048576 stripes=1024" string the
bench configuration is matched on; FETCH_DIR / WRITE_DIR are the rocprofv3
output directories of the two separate counter passes (the guide's HBM
recipe: one counter per pass).
"""
import csv
import glob
import os
import sys


def rows(d, counter, substr):
    out = []
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                name = r.get("Kernel_Name", "")
                if substr and substr not in name:
                    continue
                # rocprofv3 reports byte counters of FETCH_SIZE/WRITE_SIZE in KiB
                out.append((counter, r.get("Dispatch_Id", ""), float(r["Counter_Value"]), name))
    return out


def main():
    out, config, cmd, fdir, wdir = sys.argv[1:6]
    substr = sys.argv[6] if len(sys.argv) > 6 else "ec_encode_v16"
    recs = rows(fdir, "FETCH_SIZE", substr) + rows(wdir, "WRITE_SIZE", substr)
    if not recs:
        sys.exit("no matching counter rows")
    with open(out, "w") as f:
        f.write(f"# rocprofv3 --pmc FETCH_SIZE (pass 1) / --pmc WRITE_SIZE (pass 2) -- {cmd}\n")
        f.write(f"# config: {config} ; units KiB per dispatch; gfx950 FETCH_SIZE counts half of wide "
                "streaming reads (MI355X_MICROARCH.md HBM section): hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024\n")
        f.write("counter,dispatch,value_kib,kernel\n")
        for c, disp, v, name in recs:
            f.write(f"{c},{disp},{v:.6f},{name}\n")
    print(f"wrote {out}: {len(recs)} rows")


if __name__ == "__main__":
    main()
