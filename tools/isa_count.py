"""Static instruction mix of the sketch hash kernels' hot loop (not part of the
product).  Compiles drep_amd/csrc/sketch.hip to gfx950 assembly, finds each
kernel's unrolled loop blocks (the ones holding the BATCH-wide hash code) and
reports VALU instructions per window end.  Output feeds bench.py's VALU
roofline: python tools/isa_count.py > profiles/r03_sketch_isa.json"""
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# variant: (mangled-name pattern, k-mers/block)
KERNELS = {"default": ("k_sketch_hash21ILi64ELi2E", 2)}


def main():
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "sk.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "--cuda-device-only", "-S", "-o", asm,
                        os.path.join(ROOT, "drep_amd/csrc/sketch.hip"),
                        "-I" + os.path.join(ROOT, "drep_amd/csrc")], check=True,
                       stderr=subprocess.DEVNULL)
        s = open(asm).read()
    out = {"arch": "gfx950", "source": "drep_amd/csrc/sketch.hip", "variants": {}}
    for var, (name, per) in KERNELS.items():
        m = re.search(r"^(_ZN7drephip\d+" + name + r"\S*):", s, re.M)
        body = s[m.start():s.index(".Lfunc_end", m.start())]
        blocks, cur = [], None
        for line in body.split("\n"):
            if re.match(r"^\.LBB\S+:", line):
                cur = collections.Counter()
                blocks.append(cur)
            elif cur is not None and line.startswith("\t") and not line.strip().startswith((".", ";")):
                cur[line.strip().split()[0]] += 1
        # the hash blocks: those with the 64-bit multiply chains (mad_u64 per k-mer)
        hot = [b for b in blocks if b["v_mad_u64_u32"] >= 4 * per or
               (b["v_mad_u64_u32"] >= 3 * per and b["ds_read_b128"] >= 2 * per)]
        valu = [sum(v for k, v in b.items() if k.startswith("v_")) for b in hot]
        mul = [b["v_mul_lo_u32"] + b["v_mad_u64_u32"] + b["v_mul_hi_u32"] for b in hot]
        lds = [sum(v for k, v in b.items() if k.startswith("ds_read")) for b in hot]
        mix = collections.Counter()
        for b in hot:
            for k, v in b.items():
                if k.startswith("v_"):
                    mix[k] += v
        label = {"default": "k_sketch_hash21<64,2>"}.get(var, name)
        out["variants"][var] = {
            "kernel": label, "kmers_per_block": per, "blocks": len(hot),
            "valu_per_kmer": sum(valu) / len(hot) / per,
            "mul_per_kmer": sum(mul) / len(hot) / per,
            "lds_reads_per_kmer": sum(lds) / len(hot) / per,
            "valu_mix_per_kmer": {k: v / len(hot) / per for k, v in sorted(mix.items())},
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
