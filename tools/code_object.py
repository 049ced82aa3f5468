"""Kernel code-object inspection of a built libavz.so (CPU only, no GPU needed).

    python tools/code_object.py resources [lib.so]      per-kernel VGPR / SGPR / scratch
    python tools/code_object.py isa lib.so out.s        disassembly of the gfx950 code object
    python tools/code_object.py diff a.so b.so          kernels whose ISA differs

The gfx950 code object is unbundled from the library's .hip_fatbin section with the ROCm
LLVM tools (llvm-objcopy, clang-offload-bundler); resources come from the AMDGPU metadata
note (llvm-readelf --notes): .vgpr_count, .sgpr_count, .private_segment_fixed_size,
.group_segment_fixed_size. tests/test_code_object.py asserts that no shipped kernel uses
scratch.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
DEFAULT_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "real-time-audio-visual-zooming_amd", "avz", "libavz.so")


def extract(lib: str, out_dir: str) -> list[str]:
    """Unbundle the gfx950 code objects of `lib` (one fat binary per translation unit,
    concatenated in .hip_fatbin) into out_dir; returns their paths."""
    fat = os.path.join(out_dir, "fatbin.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib,
                    os.path.join(out_dir, "stripped.so")], check=True, capture_output=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    cos = []
    for i, a in enumerate(starts):
        part = os.path.join(out_dir, f"bundle{i}.bin")
        with open(part, "wb") as f:
            f.write(data[a:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(out_dir, f"gfx950_{i}.co")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={part}", f"--targets={TARGET}", f"--output={co}"], check=True,
                       capture_output=True)
        cos.append(co)
    return cos


def resources(lib: str = DEFAULT_LIB) -> dict[str, dict[str, int]]:
    """{kernel name: {vgpr, sgpr, agpr, scratch, lds}} from the code object's metadata note."""
    import yaml

    keys = {".vgpr_count": "vgpr", ".sgpr_count": "sgpr", ".agpr_count": "agpr",
            ".private_segment_fixed_size": "scratch", ".group_segment_fixed_size": "lds",
            ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill"}
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for co in extract(lib, d):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            doc = notes[notes.index("---"):]
            doc = doc[:doc.index("\n...")] if "\n..." in doc else doc
            meta = yaml.safe_load(doc)
            for k in meta.get("amdhsa.kernels", []):
                out[k[".name"]] = {v: int(k.get(m, -1)) for m, v in keys.items()}
    return out


def demangle(names: list[str]) -> list[str]:
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                       check=True)
    return r.stdout.splitlines()


def isa(lib: str, out: str) -> None:
    with tempfile.TemporaryDirectory() as d:
        txt = "".join(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                                      "--no-leading-addr", co], check=True, capture_output=True,
                                     text=True).stdout for co in extract(lib, d))
    with open(out, "w") as f:
        f.write(txt)


def _kernels(lib: str) -> dict[str, str]:
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "x.s")
        isa(lib, p)
        txt = open(p).read()
    blocks = re.split(r"\n(?=[0-9a-f]* ?<[^>]+>:\n)", txt)
    out = {}
    for b in blocks:
        m = re.match(r"[0-9a-f]* ?<([^>]+)>:\n", b)
        if not m:
            continue
        body = re.sub(r"<[^>]+>", "<>", b[m.end():])  # branch labels carry symbol names
        body = re.sub(r"//.*", "", body)
        out[m.group(1)] = body
    return out


def diff(a: str, b: str) -> int:
    ka, kb = _kernels(a), _kernels(b)
    # match kernels by demangled name; the round-3 synthesis kernel's 4th template argument
    # (FUSED, always false when shipped) is dropped so both generations compare
    fix = lambda n: re.sub(r"(avz_synthesis_kernel<\d+, \d+, (?:true|false)), false>", r"\1>", n)  # noqa
    da = dict(zip(map(fix, demangle(list(ka))), ka.values()))
    db = dict(zip(map(fix, demangle(list(kb))), kb.values()))
    changed = 0
    for n in sorted(set(da) | set(db)):
        if n not in da or n not in db:
            print(("only in a: " if n in da else "only in b: ") + n)
            changed += 1
        elif da[n] != db[n]:
            print(f"differs ({len(da[n].splitlines())} vs {len(db[n].splitlines())} lines): {n}")
            changed += 1
    print(f"{changed} of {len(set(da) | set(db))} functions differ")
    return changed


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "resources"
    if cmd == "resources":
        res = resources(sys.argv[2] if len(sys.argv) > 2 else DEFAULT_LIB)
        names = list(res)
        for n, d in sorted(zip(demangle(names), res.values())):
            print(f"{d.get('vgpr', -1):4d} vgpr {d.get('sgpr', -1):4d} sgpr "
                  f"{d.get('scratch', -1):5d} B scratch {d.get('lds', -1):6d} B lds  {n}")
    elif cmd == "isa":
        isa(sys.argv[2], sys.argv[3])
    elif cmd == "diff":
        sys.exit(1 if diff(sys.argv[2], sys.argv[3]) else 0)
