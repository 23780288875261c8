"""VALU per edge of the headline kernel from its ISA (test/diagnostic tool).

Compiles csrc/kern_r_f64_m2s.hip for gfx950 to assembly (the product flags of build.py), takes
rmc_kernel<double, 4, 7, 11103, 4, 256, 3> (the fused hgp_34_n1600 fp64 shot loop), and counts the
vector instructions of one variable phase (between its `s_setprio 2` / `s_setprio 0`: 7 variable
slots, 4 of degree 3 and 3 of degree 4 = 24 edge slots per thread) and of one check-phase row (the
row loop after the variable phase's barrier), by opcode and by role.  Static counts: the decision-flip
blocks (F-word xors) run only in waves where a lane's decision flipped.

    python tools/valu_breakdown.py [out.txt]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qldpc_fault_tolerance_amd.build import HIPCC_FLAGS, _hipcc  # noqa: E402

KERNEL = "_ZN5qldpc10rmc_kernelIdLi4ELi7ELi11103ELi4ELi256ELi3EEEvNS_7SMcArgsE"
ROLE = [
    (r"v_add_f64", "column sums (ldpc forward + backward adds)"),
    (r"v_mul_f64", "c2v = sel * alpha"),
    (r"v_cmp_eq_u64|v_cmp_ne_u64", "argmin test: V slot != own previous v2c"),
    (r"v_cndmask", "selects (m1 / m2 pair, decision bits)"),
    (r"v_bitop3", "c2v sign = parity ^ own sign"),
    (r"v_cmp_le_f64|v_cmp_ge_f64", "decision (w >= 0)"),
    (r"v_lshrrev_b32|v_add_u32|v_lshl_add|v_add3_u32|v_mul_lo", "addresses (F words of flipped variables, rows)"),
    (r"v_min_f64|v_max_f64", "check phase: m1 / m2"),
    (r"v_cmp_lt_f64|v_cmp_nlt_f64|v_cmp_gt_f64", "check phase: argmin compare"),
]


def counts(lines):
    c = collections.Counter()
    for t in lines:
        t = t.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            c[op] += 1
    return c


def split_conditional(lines):
    """VALU of the unconditional path vs the blocks behind `s_cbranch_execz` (decision-flip F-word
    xors, BP+OSD posterior capture): those run only in waves where some lane takes them."""
    main, cond, inside = collections.Counter(), collections.Counter(), False
    for t in lines:
        t = t.strip()
        if t.startswith("s_cbranch_execz"):
            inside = True
            continue
        if t.startswith(".LBB"):
            inside = False
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            (cond if inside else main)[op] += 1
    return main, cond


def role_of(op):
    for pat, r in ROLE:
        if re.match(pat, op):
            return r
    return "other (bit ops, moves, loop control)"


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06", "headline_sq", "valu_breakdown.txt")
    src = os.path.join(ROOT, "qldpc_fault_tolerance_amd", "csrc", "kern_r_f64_m2s.hip")
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "m2s.s")
        subprocess.run([_hipcc(), *HIPCC_FLAGS, "--offload-device-only", "-S", src, "-o", asm], check=True,
                       stderr=subprocess.DEVNULL)
        L = open(asm).read().splitlines()
    s = next(i for i, l in enumerate(L) if l.startswith(KERNEL + ":"))
    e = next(i for i in range(s, len(L)) if "s_endpgm" in L[i])
    K = L[s:e + 1]
    p2 = next(i for i, l in enumerate(K) if "s_setprio 2" in l)
    p0 = next(i for i in range(p2, len(K)) if "s_setprio 0" in K[i])
    var = counts(K[p2:p0])
    var_main, var_cond = split_conditional(K[p2:p0])
    # the check phase's row loop: the first backward branch after the variable phase's barrier
    b = next(i for i in range(p0, len(K)) if "s_barrier" in K[i])
    loop_end = next(i for i in range(b, len(K)) if re.search(r"s_cbranch_\w+ \.LBB", K[i]) and
                    any(K[j].startswith(K[i].split()[-1] + ":") for j in range(b, i)))
    label = K[loop_end].split()[-1]
    loop_start = next(j for j in range(b, loop_end) if K[j].startswith(label + ":"))
    chk = counts(K[loop_start:loop_end + 1])
    out = []
    out.append(f"kernel {KERNEL} (hgp_34_n1600 fp64 headline, 256 threads x 7 variables, D3K 4)")
    nv, nc = sum(var.values()), sum(chk.values())
    out.append(f"variable phase: {nv} VALU per thread and iteration over 24 edge slots = {nv / 24:.2f} per edge slot (static,"
               " flip blocks included)")
    by = collections.Counter()
    for op, k in var.items():
        by[role_of(op)] += k
    for r, k in by.most_common():
        out.append(f"  {k:4d}  {k / 24:5.2f}/edge  {r}")
    out.append(f"check phase row loop (one row of 7 edges: 3 x ds_read_b128 + tail): {nc} VALU = {nc / 7:.2f} per edge")
    by = collections.Counter()
    for op, k in chk.items():
        by[role_of(op)] += k
    for r, k in by.most_common():
        out.append(f"  {k:4d}  {k / 7:5.2f}/edge  {r}")
    nm, ncd = sum(var_main.values()), sum(var_cond.values())
    out.append(f"variable phase, unconditional path: {nm} VALU = {nm / 24:.2f} per edge slot; behind execz branches "
               f"(decision-flip F-word xors, posterior capture): {ncd}")
    out.append(f"static total ~ {nv / 24 + nc / 7:.1f} VALU per edge-iteration; unconditional path "
               f"{nm / 24 + nc / 7:.1f} (SQ_INSTS_VALU per edge-iteration: profiles/r06/headline_sq/)")
    out.append("by opcode, variable phase: " + ", ".join(f"{k} {v}" for k, v in var.most_common()))
    out.append("by opcode, check row: " + ", ".join(f"{k} {v}" for k, v in chk.most_common()))
    text = "\n".join(out) + "\n"
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    open(out_path, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
