"""Per-kernel ISA statistics from `hipcc --cuda-device-only -S` output: VGPRs / AGPRs, occupancy
(waves per SIMD), LDS bytes and instruction counts by class (packed / scalar fp32 FMA, fp64, MFMA,
vector memory, waits).
    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S src.hip -o out.s
    python scripts/isa_stats.py out.s [name-substring ...]
"""
import re
import sys


def kernels(text):
    starts = [m for m in re.finditer(r"^(_Z\w+):", text, flags=re.M)]
    for i, m in enumerate(starts):
        end = starts[i + 1].start() if i + 1 < len(starts) else len(text)
        yield m.group(1), text[m.start():end]


def stats(body):
    def n(p):
        return len(re.findall(p, body))

    def meta(p):
        m = re.search(p, body)
        return int(m.group(1)) if m else -1

    return dict(vgpr=meta(r"; NumVgprs:\s+(\d+)"), agpr=meta(r"; NumAgprs:\s+(\d+)"),
                occ=meta(r"; Occupancy:\s+(\d+)"), lds=meta(r"; LDSByteSize:\s+(\d+)"),
                pk_fma=n(r"\bv_pk_fma_f32"), fma=n(r"\bv_fmac?_f32"), f64=n(r"\bv_\w+_f64"),
                mfma=n(r"\bv_mfma"), vmem=n(r"\b(buffer|global)_(load|store)"), waitcnt=n(r"\bs_waitcnt\b"))


def main():
    text = open(sys.argv[1]).read()
    pats = sys.argv[2:]
    for name, body in kernels(text):
        if pats and not any(p in name for p in pats):
            continue
        s = stats(body)
        print(f"{name[:100]:100s} " + " ".join(f"{k} {v}" for k, v in s.items()))


if __name__ == "__main__":
    main()
