"""Per-phase VALU budget of the sketch hash kernel's hot loop, from the ISA
(not product code).  Compiles drep_amd/csrc/sketch.hip for gfx950 with line
tables (-gline-tables-only: the same code, plus .loc directives), walks the
k_sketch_hash21<64,2> body and attributes every instruction of the unrolled
hash blocks to the source function its .loc names -- the k-mer cut and
canonical select, the table addressing, MurmurHash3's body, fmix64, the
prefilter -- or to the loop (code-word sliding, validity, branches).  The
rare admit branch (murmur_fin, the exact test, the staging) is listed apart.
usage: python tools/isa_phases.py > profiles/r05_sketch_isa_phases.json"""
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "drep_amd/csrc/sketch.hip")


def func_ranges(lines):
    """(first, last) source lines of the functions and regions the phases name."""
    def find(pat, start=0):
        for i in range(start, len(lines)):
            if re.search(pat, lines[i]):
                return i + 1
        raise KeyError(pat)

    def body(pat):                       # a function: from its header to the closing brace at column 0
        a = find(pat)
        b = next(i + 1 for i in range(a, len(lines)) if lines[i].startswith("}"))
        return a, b
    r = {}
    r["k-mer cut + canonical select"] = (find(r"auto canon = \["), find(r"return fw <= rc"))
    r["table addressing + LDS reads"] = body(r"MEnt fetch_ent\(")
    r["Murmur body (tables combined)"] = body(r"void murmur21_ent\(")
    r["Murmur helpers (rotl, *5+c, add64, mad64)"] = None   # several functions, below
    r["fmix64 to the last multiply"] = body(r"uint64_t fmix64_q\(")
    r["prefilter (two high words, compare)"] = body(r"uint32_t prefilter_hi\(")
    r["admit branch (rare)"] = (find(r"if \(__builtin_expect\(hit, 0\)\)"), find(r"// slide one code word") - 1)
    helpers = [body(p) for p in (r"uint64_t rotl64_ab\(", r"uint64_t x5_plus\(", r"uint64_t add64\(",
                                 r"uint64_t mad64\(")]
    r["Murmur helpers (rotl, *5+c, add64, mad64)"] = helpers
    r["murmur_fin (admit branch)"] = body(r"uint64_t murmur_fin\(")
    return r


def main():
    lines = open(SRC).read().split("\n")
    ranges = func_ranges(lines)
    hit_line = next(i + 1 for i, l in enumerate(lines) if "hit |= prefilter_hi" in l)

    def phase_of(line):
        if line == hit_line:
            return "prefilter (two high words, compare)"
        for name, rg in ranges.items():
            for a, b in (rg if isinstance(rg, list) else [rg]):
                if a <= line <= b:
                    return name
        return "loop: code words, validity, control"
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "sk.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-gline-tables-only",
                        "--cuda-device-only", "-S", "-o", asm, SRC, "-I" + os.path.join(ROOT, "drep_amd/csrc")],
                       check=True, stderr=subprocess.DEVNULL)
        s = open(asm).read()
    fileno = None
    for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', s, re.M):
        if m.group(2).endswith("sketch.hip"):
            fileno = m.group(1)
    m = re.search(r"^(_ZN7drephip\d+k_sketch_hash21ILi64ELi2E\S*):", s, re.M)
    body = s[m.start():s.index(".Lfunc_end", m.start())]
    # blocks between labels; the hot ones hold the hash (2 k-mers' mad_u64 chains)
    blocks, cur, loc = [], None, 0
    for ln in body.split("\n"):
        t = ln.strip()
        if re.match(r"^\.LBB\S+:", ln):
            cur = []
            blocks.append(cur)
            continue
        lm = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if lm:
            loc = int(lm.group(2)) if lm.group(1) == fileno else 0
            continue
        if cur is None or not ln.startswith("\t") or t.startswith((".", ";")) or not t:
            continue
        cur.append((t.split()[0], loc))
    hot = [b for b in blocks if sum(1 for op, _ in b if op == "v_mad_u64_u32") >= 8]
    kmers = 2 * len(hot)
    per = collections.defaultdict(collections.Counter)
    for b in hot:
        for op, line in b:
            if op.startswith("v_"):
                per[phase_of(line)][op] += 1
    total = sum(sum(c.values()) for c in per.values())
    out = {"kernel": "k_sketch_hash21<64,2>", "source": "drep_amd/csrc/sketch.hip", "hot_blocks": len(hot),
           "kmers_in_hot_blocks": kmers, "valu_per_kmer": round(total / kmers, 3), "phases": {}}
    for name, c in sorted(per.items(), key=lambda kv: -sum(kv[1].values())):
        n = sum(c.values())
        out["phases"][name] = {"valu_per_kmer": round(n / kmers, 3), "share": round(n / total, 3),
                               "mix_per_kmer": {k: round(v / kmers, 3) for k, v in c.most_common()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
