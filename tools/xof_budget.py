#!/usr/bin/env python3
"""Per-candidate instruction budget of SampleNTT's compaction (compact_block, mlkem.hip), from the
gfx950 disassembly of the serial k_xof kernel.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S csrc/mlkem.hip -o mlkem.s
  python tools/xof_budget.py mlkem.s [K]

The main pass of k_xof is one loop iteration per SHAKE128 block: the Keccak permutation (its own
loop, 2 rounds per iteration) then the compaction of the block's 14 triplets (8 candidates each).
Every instruction between the end of the Keccak loop and the block loop's back-edge is classified
by role; each triplet's two branches (the pending chunk's flush, the completed chunk's ring reads)
run for the whole wave whenever any of its 64 lanes needs them, so they are counted once per
triplet like the straight-line part.  Output: one JSON object (per block, per triplet, per
candidate), the Keccak loop's counts alongside."""
import json
import re
import sys
from collections import Counter

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
key = f"_ZN3qrk5mlkem6k_roleINS0_4RXofILi{K}ELb0EEEEEvT_:"
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(key))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = []
for l in lines[start:end]:
    s = l.split(";")[0].strip()  # drop trailing comments (loop-header notes on labels)
    if not s or s.startswith(";") or (s.startswith(".") and not s.endswith(":")):
        continue
    body.append(s)

# the Keccak round loop: the first backward s_cbranch_scc1 whose target label precedes it
labels = {s[:-1]: i for i, s in enumerate(body) if s.endswith(":")}
loops = []
for i, s in enumerate(body):
    m = re.match(r"s_cbranch_\w+ (\.LBB\w+)", s) or re.match(r"s_branch (\.LBB\w+)", s)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        loops.append((labels[m.group(1)], i))
kloop = min(loops, key=lambda x: x[1] - x[0])  # the innermost loop: the Keccak rounds
bloop = max(loops, key=lambda x: x[1] - x[0])  # the block loop
keccak = [s for s in body[kloop[0]:kloop[1] + 1] if not s.endswith(":")]
compact = [s for s in body[kloop[1] + 1:bloop[1] + 1] if not s.endswith(":")]


def role(s: str) -> str:
    op = s.split()[0]
    if op.startswith("ds_write"):
        return "ring_write (LDS)"
    if op.startswith("ds_read"):
        return "ring_read (LDS)"
    if op.startswith(("global_store", "flat_store", "buffer_store")):
        return "chunk_store (VMEM)"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait/nop"
    if op.startswith("s_"):
        return "scalar/branch"
    if op == "v_bitop3_b32" and "bitop3:0xea" in s:
        return "address (bitop3)"
    if op == "v_cmp_gt_u32_e32" or op == "v_cndmask_b32_e32":
        return "accept/count"
    if op == "v_add_u32_e32":
        return "accept/count"
    if op in ("v_bfe_u32", "v_alignbit_b32", "v_perm_b32") or (op == "v_and_b32_e32" and "0xfff," in s) or \
            (op == "v_lshrrev_b32_e32" and s.split()[2] == "20,"):
        return "split12"
    if op in ("v_ashrrev_i32_e32", "v_cmp_ne_u32_e32", "v_cmp_gt_i32_e64", "v_cmp_lt_i32_e32"):
        return "chunk_check"
    if op in ("v_mad_u64_u32", "v_lshl_add_u64") or (op == "v_and_b32_e32" and ("0x7fffffc0" in s or " 1," in s)) or \
            (op == "v_lshlrev_b32_e32" and s.split()[2] == "5,") or (op == "v_and_b32_e32" and "0x800" in s):
        return "flush_address"
    if op in ("v_lshlrev_b32_e32", "v_lshrrev_b32_e32", "v_or_b32_e32", "v_or3_b32", "v_lshl_or_b32"):
        return "flush_pack"
    if op == "v_mov_b32_e32":
        return "register_move"
    return "other:" + op


c = Counter(role(s) for s in compact)
valu = sum(v for k, v in c.items() if not k.endswith(("(LDS)", "(VMEM)")) and k not in ("wait/nop", "scalar/branch"))
kvalu = sum(1 for s in keccak if s.startswith("v_"))
out = {
    "source": "k_role<RXof<%d,false>> (serial k_xof), gfx950 -O3 disassembly" % K,
    "keccak_loop": {"instructions_per_iteration": len(keccak), "valu_per_iteration": kvalu,
                    "iterations_per_permutation": 12, "valu_per_permutation": 12 * kvalu,
                    "algorithmic_ops_per_permutation": 4320},
    "compaction_per_block": dict(sorted(c.items(), key=lambda kv: -kv[1])),
    "compaction_valu_per_block": valu,
    "compaction_valu_per_triplet": round(valu / 14, 1),
    "compaction_valu_per_candidate": round(valu / 112, 2),
    "valu_per_block_total": 12 * kvalu + valu,
    "algorithmic_over_issued_model": round(4320 / (12 * kvalu + valu), 3),
}
print(json.dumps(out, indent=1))
