"""Priced model of the sketch hash kernel (k_sketch_hash21<64,2>) against its
measured time -- not part of the product.

Inputs (one GPU call, tools/gpu_round.sh STEPS=price):
  valu_microbench_<r>.json  tools/valu_microbench.hip: wall time per wave64
                            instruction per SIMD at 8 waves/SIMD, per class
  sketch_ms_<r>.json        tools/sketch_ablate.py: the hash kernel's time at
                            configs[1] (1000 synthetic 5 Mbp genomes, first round)
The hot loop's static mix is counted here from the current source (gfx950
assembly, the unrolled hash blocks: tools/isa_count.py's selection), every
instruction is priced at its class's measured rate, and the sum over one k-mer
times the k-mers per SIMD is the predicted time.

usage: python tools/sketch_priced.py <dir with the GPU outputs> > profiles/r06_sketch_priced.json
"""
import collections
import glob
import json
import os
import re
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WINDOW_ENDS = 5_013_504_000          # configs[1]: window ends per launch (profiles/r05_sketch_ablation.json)
SIMDS = 1024

# hot-loop mnemonic -> microbench class (tools/valu_microbench.hip `ops` names)
CLASS = {
    "v_xor_b32_e32": "v_xor_b32_e32", "v_add_u32_e32": "v_add_u32_e32", "v_add3_u32": "v_add3_u32",
    "v_alignbit_b32": "v_alignbit_b32", "v_and_b32_e32": "v_and_b32_e32 (literal)", "v_bfi_b32": "v_bfi_b32",
    "v_bfrev_b32_e32": "v_bfrev_b32_e32", "v_cmp_ge_u32_e32": "v_cmp_ge_u32_e32 (vcc)",
    "v_cmp_lt_u32_e32": "v_cmp_ge_u32_e32 (vcc)", "v_cmp_lt_u64_e32": "v_cmp_lt_u64_e32 (vcc)",
    "v_cndmask_b32_e32": "v_cndmask_b32_e32 (vcc)", "v_lshl_add_u64": "v_lshl_add_u64",
    "v_lshlrev_b32_e32": "v_lshlrev_b32_e32", "v_lshlrev_b32_sdwa": "v_lshlrev_b32_sdwa (sgpr shift, byte select)",
    "v_or_b32_sdwa": "v_lshlrev_b32_sdwa (sgpr shift, byte select)", "v_lshlrev_b64": "v_lshlrev_b64",
    "v_lshrrev_b32_e32": "v_lshrrev_b32_e32", "v_lshrrev_b64": "v_lshrrev_b64", "v_mad_u64_u32": "v_mad_u64_u32",
    "v_min_u32_e32": "v_min_u32_e32", "v_mov_b32_e32": "v_mov_b32_e32", "v_mov_b64_e32": "v_mov_b64_e32",
    "v_mul_hi_u32": "v_mul_hi_u32", "v_mul_lo_u32": "v_mul_lo_u32", "v_not_b32_e32": "v_not_b32_e32",
    "v_or_b32_e32": "v_or_b32_e32", "v_perm_b32": "v_perm_b32",
}
SELECT = "select: v_cmp_lt_u64_e32 vcc + 2 v_cndmask_b32_e32"


def hot_mix():
    """Instructions per k-mer of the hot loop, every kind (VALU, LDS, SALU, waits)."""
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "sk.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", "-o", asm, os.path.join(ROOT, "drep_amd/csrc/sketch.hip"),
                        "-I" + os.path.join(ROOT, "drep_amd/csrc")], check=True, stderr=subprocess.DEVNULL)
        s = open(asm).read()
    m = re.search(r"^(_ZN7drephip\d+k_sketch_hash21ILi64ELi2E\S*):", s, re.M)
    body = s[m.start():s.index(".Lfunc_end", m.start())]
    blocks, cur = [], None
    for line in body.split("\n"):
        if re.match(r"^\.LBB\S+:", line):
            cur = collections.Counter()
            blocks.append(cur)
        elif cur is not None and line.startswith("\t") and not line.strip().startswith((".", ";")):
            cur[line.strip().split()[0]] += 1
    per = 2                                                   # k-mers per hash block (BATCH)
    hot = [b for b in blocks if b["v_mad_u64_u32"] >= 4 * per or
           (b["v_mad_u64_u32"] >= 3 * per and b["ds_read_b128"] >= 2 * per)]
    tot = collections.Counter()
    for b in hot:
        tot.update(b)
    return {k: v / len(hot) / per for k, v in sorted(tot.items())}, len(hot)


def main():
    d = sys.argv[1]
    mbs = [json.load(open(f)) for f in sorted(glob.glob(os.path.join(d, "valu_microbench_*.json")))]
    sks = [json.load(open(f)) for f in sorted(glob.glob(os.path.join(d, "sketch_ms_*.json")))]
    price = {}                                                # class -> [ns per wave-inst per SIMD] over reps
    clock = {}
    for mb in mbs:
        for r in mb["results"]:
            price.setdefault(r["inst"], []).append(r["ns_per_wave_inst_per_simd"])
            clock.setdefault(r["inst"], []).append(r["clock_ghz"])
    p = {k: statistics.median(v) for k, v in price.items()}
    ghz = {k: statistics.median(v) for k, v in clock.items()}
    mix, nblocks = hot_mix()
    rows = []
    total_ns = 0.0
    # the canonical select: every v_cmp_lt_u64 + its two v_cndmask, priced as the
    # measured three-instruction sequence (per instruction: p[SELECT])
    nsel = min(mix.get("v_cndmask_b32_e32", 0) / 2, mix.get("v_cmp_lt_u64_e32", 0))
    left = dict(mix)
    if nsel:
        left["v_cndmask_b32_e32"] -= 2 * nsel
        left["v_cmp_lt_u64_e32"] -= nsel
        c = 3 * nsel * p[SELECT]
        rows.append({"class": SELECT, "per_kmer": 3 * nsel, "ns_per_wave_inst": p[SELECT], "ns_per_kmer_wave": c})
        total_ns += c
    unpriced = {}
    for k, n in sorted(left.items()):
        if not k.startswith("v_") or n <= 1e-9:
            continue
        cls = CLASS.get(k)
        if cls is None or cls not in p:
            unpriced[k] = n
            continue
        c = n * p[cls]
        rows.append({"mnemonic": k, "class": cls, "per_kmer": n, "ns_per_wave_inst": p[cls], "ns_per_kmer_wave": c})
        total_ns += c
    valu_n = sum(n for k, n in mix.items() if k.startswith("v_"))
    # LDS reads and SALU inside a VALU-bound stream: their measured marginal cost
    xor = p["v_xor_b32_e32"]
    lds_extra = (p["mixed: 64 v_xor_b32 + 2 ds_read_b128 + 3 ds_read_b64 (per v_xor)"] -
                 p["control for 33: the same loop without the LDS reads (per v_xor)"]) * 64 / 5
    salu_extra = (p["mixed: 64 v_xor_b32 + 4 s_mov_b32 (per v_xor)"] - xor) * 64 / 4
    n_lds = sum(n for k, n in mix.items() if k.startswith("ds_read"))
    n_salu = sum(n for k, n in mix.items() if k.startswith("s_") and k not in ("s_waitcnt", "s_nop", "s_barrier")
                 and not k.startswith("s_cbranch"))
    lds_ns = n_lds * max(lds_extra, 0.0)
    salu_ns = n_salu * max(salu_extra, 0.0)
    # the LDS pipe alone (every SIMD of the CU reading, as in the microbench): 2 b128 + 3 b64 per k-mer
    lds_pipe_ns = (mix.get("ds_read_b128", 0) * p["ds_read_b128, random 16-B entry of 256 (4 KiB)"] +
                   mix.get("ds_read_b64", 0) * p["ds_read_b64, random 8-B entry of 256 (2 KiB)"])
    units = WINDOW_ENDS / 64 / SIMDS                          # k-mer waves per SIMD
    pred_valu_ms = units * total_ns * 1e-6
    pred_ms = units * (total_ns + lds_ns + salu_ns) * 1e-6
    meas = [s["hash_ms_median"] for s in sks]
    meas_ms = statistics.median(meas) if meas else None
    out = {
        "kernel": "k_sketch_hash21<64,2>",
        "workload": "configs[1]: 1000 synthetic 5 Mbp genomes, k=21, s=1000 (first threshold round)",
        "window_ends_per_launch": WINDOW_ENDS,
        "method": ("every instruction of the hot loop (static mix per k-mer, counted from the gfx950 assembly of "
                   "drep_amd/csrc/sketch.hip) priced at its class's measured wall time per wave64 instruction per "
                   "SIMD with 8 waves on every SIMD (tools/valu_microbench.hip, 8 independent chains per lane); "
                   "the canonical select priced as its measured 3-instruction sequence; LDS reads and SALU at their "
                   "measured marginal cost inside a VALU-bound stream; predicted ms = sum x window ends / 64 / 1024 "
                   "SIMDs"),
        "microbench_reps": len(mbs), "sketch_reps": len(sks),
        "microbench_clock_ghz_median": statistics.median(ghz.values()) if ghz else None,
        "hot_blocks": nblocks,
        "valu_per_kmer": valu_n,
        "lds_reads_per_kmer": n_lds, "salu_per_kmer": n_salu,
        "mix_per_kmer": mix,
        "priced_valu": sorted(rows, key=lambda r: -r["ns_per_kmer_wave"]),
        "unpriced": unpriced,
        "valu_ns_per_kmer_wave": total_ns,
        "valu_ns_per_instruction_avg": total_ns / valu_n,
        "lds_marginal_ns_per_read": lds_extra, "salu_marginal_ns_per_instr": salu_extra,
        "lds_pipe_alone_ns_per_kmer_wave_per_simd": lds_pipe_ns,
        "lds_pipe_alone_ms": units * lds_pipe_ns * 1e-6,
        "predicted_valu_only_ms": pred_valu_ms,
        "predicted_ms": pred_ms,
        "measured_hash_ms": meas_ms, "measured_reps_ms": meas,
        "predicted_over_measured": pred_ms / meas_ms if meas_ms else None,
        "prices_ns": p, "prices_clock_ghz": ghz,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
