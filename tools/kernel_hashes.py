#!/usr/bin/env python3
"""Per-kernel disassembly hashes of the default build's device code.

    tools/kernel_hashes.py [--csrc DIR] OUT.json

Compiles every csrc/*.hip device-only for gfx950 (the Makefile's flags), disassembles the code
objects and hashes each function's instruction text (addresses and branch-target labels
normalised), so a source clean-up can be shown to leave every remaining kernel bit-identical.
Compare two runs with `tools/kernel_hashes.py --diff A.json B.json`.
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

LLVM = "/opt/rocm/lib/llvm/bin"


def build(csrc, tmp, f):
    b = os.path.join(tmp, f + ".bundle")
    co = os.path.join(tmp, f + ".co")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-w",
                    "--cuda-device-only", "-c", os.path.join(csrc, f), "-o", b], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}"], check=True)
    return co


def functions(co):
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                         check=True, capture_output=True, text=True).stdout
    out, name, body = {}, None, []
    pc = 0  # instructions since the last s_getpc_b64: their literals are PC-relative offsets
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]* ?<(.+)>:$", line.strip())
        if m:
            if name:
                out[name] = body
            name, body = m.group(1), []
        elif name and line.strip() and line.strip() != "...":
            ins = re.sub(r"<[^>]*>", "<L>", re.sub(r"//.*$", "", line)).strip()
            if ins.startswith("s_getpc_b64"):
                pc = 16
            elif pc:
                pc -= 1
                if ins.startswith(("s_add_u32", "s_addc_u32", "s_add_co_u32", "s_addc_co_u32")):
                    ins = re.sub(r"0x[0-9a-fA-F]+|\b\d+\b", "#", ins)
            body.append(ins)
    if name:
        out[name] = body
    return {k: hashlib.sha256("\n".join(v).encode()).hexdigest()[:16] for k, v in out.items()}


def main():
    a = sys.argv[1:]
    if a and a[0] == "--diff":
        x, y = json.load(open(a[1])), json.load(open(a[2]))
        same = sorted(k for k in x if k in y and x[k] == y[k])
        changed = sorted(k for k in x if k in y and x[k] != y[k])
        gone = sorted(k for k in x if k not in y)
        new = sorted(k for k in y if k not in x)
        print(json.dumps({"identical": len(same), "changed": changed, "removed": gone, "added": new}, indent=1))
        return
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "quantum-resistant-p2p_amd", "csrc")
    if a and a[0] == "--csrc":
        csrc, a = a[1], a[2:]
    with tempfile.TemporaryDirectory() as tmp:
        srcs = sorted(f for f in os.listdir(csrc) if f.endswith(".hip"))
        with ThreadPoolExecutor(8) as ex:
            cos = list(ex.map(lambda f: build(csrc, tmp, f), srcs))
        res = {}
        for f, co in zip(srcs, cos):
            for k, h in functions(co).items():
                res[f"{f}:{k}"] = h
    json.dump(res, open(a[0], "w"), indent=1, sort_keys=True)
    print(f"{len(res)} functions -> {a[0]}")


if __name__ == "__main__":
    main()
