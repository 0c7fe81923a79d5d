"""Compile one kernel source to gfx950 assembly and summarise each kernel:
VGPR / AGPR / scratch use, main-loop and post-loop instruction mix.

  python tools/isa_stats.py csrc/kernels/gemmt.hip --match gemmt_kernelILb0ELb0ELi0ELi0ELi0ELi0E

Used to iterate on register allocation and epilogue code without a GPU.
"""
import argparse
import collections
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def compile_asm(src, out):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           "-munsafe-fp-atomics", "-I" + os.path.join(ROOT, "csrc", "kernels"), src, "-o", out]
    subprocess.run(cmd, check=True)


def kernels(lines):
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            j = next(k for k in range(i, len(lines)) if lines[k].strip().startswith("s_endpgm"))
            yield m.group(1), i, j


def meta(text, name):
    i = text.find(".amdhsa_kernel " + name)
    if i < 0:
        return {}
    j = text.find(".end_amdhsa_kernel", i)
    out = {}
    for l in text[i:j].split("\n"):
        p = l.split()
        if len(p) == 2 and p[0] in (".amdhsa_next_free_vgpr", ".amdhsa_accum_offset",
                                    ".amdhsa_private_segment_fixed_size"):
            out[p[0].split("_", 1)[1]] = int(p[1])
    return out


def summarise(lines, st, end):
    body = lines[st:end + 1]
    ins = lambda seg: [l.split()[0] for l in seg if l.startswith("\t") and not l.strip().startswith((";", "."))]
    hdr = [i for i, l in enumerate(body) if "Inner Loop Header" in l]
    if not hdr:
        return {"total": len(ins(body))}
    h = hdr[-1]
    lab = body[h].split(":")[0]
    e = next((i for i, l in enumerate(body) if "s_cbranch" in l and l.strip().endswith(lab)), None)
    loop = ins(body[h:e + 1]) if e else []
    post = ins(body[e + 1:]) if e else []
    return {"loop": len(loop), "loop_mix": collections.Counter(loop).most_common(12), "post": len(post),
            "post_mix": collections.Counter(post).most_common(16)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--match", default="")
    ap.add_argument("--out", default="/tmp/isa_stats.s")
    ap.add_argument("--no-compile", action="store_true")
    a = ap.parse_args()
    if not a.no_compile:
        compile_asm(a.src, a.out)
    text = open(a.out).read()
    lines = text.split("\n")
    for name, st, end in kernels(lines):
        if a.match not in name:
            continue
        print(name, meta(text, name))
        for k, v in summarise(lines, st, end).items():
            print("   ", k, v)


if __name__ == "__main__":
    sys.exit(main())
