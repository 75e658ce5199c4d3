"""The sketch hash kernel's binding resource, as one JSON (not product code):
per variant of tools/gpu_r05_sketch_ablate.sh, the hot loop's VALU
instructions per window end (this tool compiles sketch.hip for gfx950 with the
variant's flags and counts the unrolled hash blocks, as tools/isa_phases.py
does) next to the hash kernel's same-box time (gpurun_out/r05skabl/*.json),
and the SIMD-cycles each wave64 VALU instruction took:

    cycles / wave-instruction / SIMD = t x 2.4 GHz x 1024 SIMDs / (VALU per window end x window ends / 64)

The no-LDS build (no table reads: the entries come from the k-mer's own words)
is this instruction stream with nothing but VALU and its code-word loads: its
per-instruction cost is the floor the product is compared with.

usage: python tools/sketch_ablation_json.py gpurun_out/r05skabl > profiles/r05_sketch_ablation.json"""
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "drep_amd/csrc/sketch.hip")
N, L, P_TILE = 1000, 5_000_000, 32768          # configs[1] (tools/sketch_ablate.py)
VARIANTS = {   # name: (hipcc flags, library, DREPHIP_SK_KMASK)
    "product": ([], "default", None),
    "real": (["-DDREPHIP_SK_ABLATE=1"], "lib_ab/skabl", "0x3FF"),
    "bcast": (["-DDREPHIP_SK_ABLATE=1"], "lib_ab/skabl", "0"),
    "nolds": (["-DDREPHIP_SK_ABLATE=2"], "lib_ab/sknolds", None),
}


def valu_per_window_end(flags):
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "sk.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", "-o", asm, SRC, "-I" + os.path.join(ROOT, "drep_amd/csrc")] + flags,
                       check=True, stderr=subprocess.DEVNULL)
        s = open(asm).read()
    m = re.search(r"^(_ZN7drephip\d+k_sketch_hash21ILi64ELi2E\S*):", s, re.M)
    body = s[m.start():s.index(".Lfunc_end", m.start())]
    blocks, cur = [], None
    for ln in body.split("\n"):
        if re.match(r"^\.LBB\S+:", ln):
            cur = collections.Counter()
            blocks.append(cur)
        elif cur is not None and ln.startswith("\t") and not ln.strip().startswith((".", ";")) and ln.strip():
            cur[ln.strip().split()[0]] += 1
    hot = [b for b in blocks if b["v_mad_u64_u32"] >= 8]       # two k-mers' multiply chains per block
    valu = sum(v for b in hot for k, v in b.items() if k.startswith("v_"))
    lds = sum(v for b in hot for k, v in b.items() if k.startswith("ds_read"))
    return valu / (2 * len(hot)), lds / (2 * len(hot))


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out/r05skabl")
    padded = -(-(L + 1) // P_TILE) * P_TILE
    window_ends = N * padded
    out = {"kernel": "k_sketch_hash21<64,2>", "workload": "configs[1]: 1000 synthetic 5 Mbp genomes, first threshold round",
           "timing": "HIP events, median of 10 launches per rep, reps interleaved on one box (tools/gpu_r05_sketch_ablate.sh)",
           "window_ends_per_launch": window_ends, "clock_ghz_nominal": 2.4, "simds": 1024, "variants": {}}
    for name, (flags, lib, kmask) in VARIANTS.items():
        reps = [json.load(open(f)) for f in sorted(glob.glob(os.path.join(d, name + ".*.json")))]
        if not reps:
            continue
        ms = float(np.median([r["hash_ms_median"] for r in reps]))
        v, lds = valu_per_window_end(flags)
        wi = v * window_ends / 64
        out["variants"][name] = {"hipcc_flags": flags, "library": lib, "kmask": kmask, "hash_ms": round(ms, 4),
                                 "valu_per_window_end": round(v, 3), "lds_reads_per_window_end": round(lds, 3),
                                 "cycles_per_wave_inst_per_simd": round(ms * 1e-3 * 2.4e9 * 1024 / wi, 4),
                                 "reps_ms": [round(r["hash_ms_median"], 4) for r in reps]}
    V = out["variants"]
    if "product" in V and "nolds" in V:
        fl, pr = V["nolds"]["cycles_per_wave_inst_per_simd"], V["product"]["cycles_per_wave_inst_per_simd"]
        out["floor"] = {"cycles_per_wave_inst_per_simd": fl,
                        "product_ms_at_floor": round(fl * V["product"]["valu_per_window_end"] * window_ends / 64 /
                                                     (2.4e9 * 1024) * 1e3, 4),
                        "product_frac_of_floor_rate": round(fl / pr, 4),
                        "note": "the no-LDS build's per-instruction cost x the product's VALU count: the time the "
                                "product's own instruction stream takes with no table reads at all"}
    if "real" in V and "bcast" in V:
        out["lds_bank_conflicts_cost"] = round(V["real"]["hash_ms"] / V["bcast"]["hash_ms"] - 1, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
