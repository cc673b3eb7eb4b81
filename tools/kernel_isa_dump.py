"""Dump the gfx950 ISA of every kernel in libbolt_mi355x.so, normalised so two
builds compare by content: one file per kernel symbol with addresses, raw
encodings and branch-target comments removed (branch offsets stay: they are
relative, so an identical body has identical offsets).

    python tools/kernel_isa_dump.py bolt_amd/libbolt_mi355x.so OUTDIR
    diff -r OUTDIR_before OUTDIR_after        (no output: the same kernels, instruction for instruction)

Used to show that stripping the rejected A/B variants from the kernel sources
changed no shipped kernel (VERDICT r04 Next #5)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so, tmp):
    """The gfx950 code object of every translation unit: .hip_fatbin holds
    one offload bundle per source file with device code (each starts with the
    magic, then uint64 entry count and per entry uint64 offset / size /
    triple length + triple, offsets from the bundle's start)."""
    import struct
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, so,
                    os.path.join(tmp, "stripped.so")], check=True)
    data = open(fat, "rb").read()
    out = []
    for i, m in enumerate(re.finditer(re.escape(MAGIC), data)):
        base = m.start()
        p = base + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if triple.endswith("gfx950"):
                co = os.path.join(tmp, "gfx950_%d.co" % i)
                open(co, "wb").write(data[base + off:base + off + size])
                out.append(co)
    return out


def kernels(co):
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                         check=True, capture_output=True, text=True).stdout
    cur, body, res = None, [], {}
    for ln in out.splitlines():
        m = re.match(r"^([A-Za-z_][\w.$]*)>?:\s*$", ln.strip("<"))
        if m and not ln.startswith(" ") and not ln.startswith("\t"):
            if cur:
                res[cur] = body
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        s = ln.split("//")[0].strip()
        if s:
            body.append(re.sub(r"\s+", " ", s))
    if cur:
        res[cur] = body
    return res


def main():
    so, outdir = sys.argv[1], sys.argv[2]
    os.makedirs(outdir, exist_ok=True)
    ks = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(so, tmp):
            for name, body in kernels(co).items():
                assert name not in ks, name
                ks[name] = body
    for name, body in ks.items():
        with open(os.path.join(outdir, name[:200] + ".s"), "w") as f:
            f.write("\n".join(body) + "\n")
    print("%d symbols, %d instructions -> %s" % (len(ks), sum(len(b) for b in ks.values()), outdir))


if __name__ == "__main__":
    main()
