"""HBM traffic per launch of the sketch hash kernel from rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE in separate runs; tools/profile_round.sh), with the
MI355X_MICROARCH.md HBM corrections: counters are KB; on gfx950 FETCH_SIZE
tallies 128-B read requests at 64 B, so reads are doubled (consistent here:
undoubled reads would be half the bytes the kernel must touch).  Not part of
the product.

usage: python tools/traffic_json.py <round_dir> <genomes_per_launch> <genome_bp> > profiles/<round>_sketch_traffic.json
"""
import csv
import json
import os
import sys

KERNEL = "k_sketch_hash21"


def per_dispatch(path, counter):
    rows = list(csv.DictReader(open(path)))
    vals = {}
    for r in rows:
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values()), {r["Kernel_Name"] for r in rows if KERNEL in r["Kernel_Name"]}


def main():
    d, G, L = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    tile = 32768
    P = ((L + 1 + tile - 1) // tile) * tile               # padded span of one single-record genome
    f, names = per_dispatch(os.path.join(d, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), "FETCH_SIZE")
    w, _ = per_dispatch(os.path.join(d, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), "WRITE_SIZE")
    fetch_kb, write_kb = sum(f) / len(f), sum(w) / len(w)
    alg = G * P * 3 / 8
    hbm = 2 * fetch_kb * 1024 + write_kb * 1024
    from drep_amd import _lib
    print(json.dumps({
        "kernel": sorted(names)[0] if names else KERNEL,
        "build_id": _lib.build_id(),
        "command": "rocprofv3 --pmc <C> -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 (one pass per counter)",
        "dispatches": [len(f), len(w)],
        "genomes_per_launch": G,
        "bases_per_launch": G * P,
        "fetch_size_kb": fetch_kb,
        "write_size_kb": write_kb,
        "algorithmic_bytes_per_launch": alg,
        "hbm_bytes_per_launch": hbm,
        "correction": "MI355X_MICROARCH.md HBM: FETCH_SIZE/WRITE_SIZE are KB; on gfx950 FETCH_SIZE reads 1/2 of "
                      "the bytes of a coalesced stream, so reads are doubled; writes (set-insert atomics) as is",
        "read_over_algorithmic": 2 * fetch_kb * 1024 / alg,
    }, indent=1))


if __name__ == "__main__":
    main()
