"""Issue-time model of lk_multi_kernel's VALU mix (round 5).

gfx950 issues VALU instructions at two rates (profiles/r05/a_valu_rates*.txt, measured
with tools/valu_rates*.hip: 4 waves per SIMD, 8 independent chains each): the "fast"
class -- 32-bit integer add / sub, logic, mov, right shifts, f32 add / sub / mul / fma --
at ~1.0-1.3 ns per wave-instruction per SIMD (2 cycles at 2.4 GHz: the 1,228.8 G
wave-instructions/s peak), everything else measured (dot2 / dot4, perm, left shift,
add3, cndmask, cmp, cvt, floor, DPP, mul_lo / mul_24, packed f32, f64) at ~1.75-2.0 ns
(4 cycles). A kernel's attainable VALU rate is therefore set by its mix.

This tool reads the compiled ISA of the temporal LK kernel, weights each basic block by
how often a wave executes it (prologue / epilogue once, the level loop's blocks per
level, the trip loop's per iteration; the trip loop's re-staging path -- blocks with LDS
stores or the staging loop -- as rare), classifies every VALU instruction by the measured
table, and prints the predicted VALU per wave (to compare with SQ_INSTS_VALU / SQ_WAVES),
the slow-class share and the mix-weighted peak rate:

    peak_mix = 1024 SIMDs / (sum over instructions of weight x ns) x (sum of weights)

Usage: python tools/lk_mix_model.py [--asm FILE] [--levels 4] [--iters 16.5]
(--iters: trip-loop iterations per wave over all levels, i.e. the slowest of its four
features per level; the bench's lk_iterations / features x the max-of-4 factor.)
"""
import argparse
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "lk_multi_kernelILi4ELi1ELi3ELi2ELi21ELi21ELi7E"

# ns per wave-instruction per SIMD (4 waves / SIMD), profiles/r05/a_valu_rates*.txt
FAST_NS = 1.12
SLOW_NS = 1.82
FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32",
        "v_fmac_f32", "v_fma_f32", "v_mac_f32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_mov_b32",
        "v_lshrrev_b32", "v_ashrrev_i32", "v_not_b32"}
# readlane / readfirstlane write an SGPR (VALU issue all the same): slow class assumed
NOT_VALU = ("v_nop",)


def base_op(mn):
    mn = re.sub(r"_e(32|64)$", "", mn)
    mn = re.sub(r"_(dpp|sdwa)$", "_dpp", mn)
    return mn


def cls(op):
    if op.endswith("_dpp"):
        return "slow"
    return "fast" if op in FAST else "slow"


def kernel_asm(path, kernel=None):
    KERNEL = kernel or globals()["KERNEL"]
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith("_Z") and KERNEL in l and l.rstrip().endswith(":")
                 or (l.startswith("_Z") and KERNEL in l.split(":")[0]))
    end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
    return text[start:end + 1]


def blocks(lines):
    """(label, depth, rare, [instruction mnemonics]) per basic block."""
    out = []
    cur = {"label": "entry", "depth": 0, "ins": [], "rare": False}
    pend_depth = None
    for l in lines:
        s = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):|^; %bb\.(\d+):", s)
        if m:
            out.append(cur)
            cur = {"label": m.group(1) or f"bb.{m.group(2)}", "depth": 0, "ins": [], "rare": False}
            ds = [int(x) for x in re.findall(r"Depth=(\d+)", s)]
            cur["depth"] = max(ds) if ds else 0
            continue
        if s.startswith(";") and "Depth=" in s and not cur["ins"]:
            cur["depth"] = max([cur["depth"]] + [int(x) for x in re.findall(r"Depth=(\d+)", s)])
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        mn = s.split()[0]
        cur["ins"].append(mn)
    out.append(cur)
    for b in out:
        b["rare"] = b["depth"] >= 3 or (b["depth"] == 2 and any(i.startswith("ds_write") or i.startswith("ds_bpermute")
                                                                 for i in b["ins"]))
    # round 6: the single-group tail's loop (depth 2 again after the trip loop's blocks and
    # the depth-1 tail entry) runs the wave's single-group iterations only
    seen2 = back1 = False
    for b in out:
        if b["depth"] >= 2 and not back1:
            seen2 = True
        elif b["depth"] == 1 and seen2:
            back1 = True
        b["tail"] = back1 and b["depth"] >= 2
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=None)
    ap.add_argument("--levels", type=float, default=4.0)
    ap.add_argument("--iters", type=float, default=14.9, help="group-path trip-loop iterations per wave")
    ap.add_argument("--tail-iters", type=float, default=1.6,
                    help="single-group tail iterations per wave (oracle replay: 9.8 %% of the headline's wave "
                         "iterations are single-group, profiles/r05/i_lk_iter_waste.txt)")
    ap.add_argument("--rare", type=float, default=0.05, help="re-staging executions per iteration")
    ap.add_argument("--kernel", default=KERNEL, help="mangled-name fragment of the instance")
    ap.add_argument("--json", default=None, help="write the result here (bench.py reads profiles/lk_issue_model.json)")
    a = ap.parse_args()
    path = a.asm
    if path is None:
        path = "/tmp/lk_mix_model.s"
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", f"-I{REPO}/include",
               f"-I{REPO}/svo_amd/csrc", "--offload-arch=gfx950", "--cuda-device-only", "-S",
               f"{REPO}/svo_amd/csrc/lk.hip", "-o", path]
        subprocess.run(cmd, check=True)
    bl = blocks(kernel_asm(path, a.kernel))
    w_of = {0: 1.0, 1: a.levels, 2: a.iters}
    tot_n = tot_ns = 0.0
    by_cls = {"fast": 0.0, "slow": 0.0}
    by_depth = {}
    for b in bl:
        w = w_of.get(min(b["depth"], 2), 1.0)
        if b.get("tail"):
            w = a.tail_iters
        if b["rare"]:
            w = (a.tail_iters if b.get("tail") else a.iters) * a.rare
        for mn in b["ins"]:
            if not mn.startswith("v_") or mn.startswith(NOT_VALU):
                continue
            op = base_op(mn)
            c = cls(op)
            tot_n += w
            tot_ns += w * (FAST_NS if c == "fast" else SLOW_NS)
            by_cls[c] += w
            by_depth[b["depth"]] = by_depth.get(b["depth"], 0.0) + w
    ns_per = tot_ns / tot_n
    peak_mix = 1024 / ns_per  # G wave-instructions / s over 1,024 SIMDs
    print(f"predicted VALU per wave {tot_n:.0f} (by loop depth: "
          + ", ".join(f"{d}: {v:.0f}" for d, v in sorted(by_depth.items())) + ")")
    print(f"slow-class share {by_cls['slow'] / tot_n:.3f}; mean {ns_per:.3f} ns per wave-instruction per SIMD")
    print(f"mix-weighted VALU peak {peak_mix:.1f} G wave-instr/s (fast-class peak 1228.8; all-fast at "
          f"{FAST_NS} ns: {1024 / FAST_NS:.1f})")
    if a.json:
        import json
        json.dump({"kernel": "lk_multi_kernel<4, 1, 3, 2, 21, 21, 7, false>", "predicted_valu_per_wave": round(tot_n),
                   "slow_share": round(by_cls["slow"] / tot_n, 4), "ns_per_instr": round(ns_per, 4),
                   "peak_mix_G": round(peak_mix, 1), "fast_ns": FAST_NS, "slow_ns": SLOW_NS,
                   "levels": a.levels, "iters_per_wave": a.iters, "tail_iters_per_wave": a.tail_iters,
                   "source": "tools/lk_mix_model.py: the compiled ISA's VALU instructions weighted by block "
                             "frequency, priced at the measured per-class rates (profiles/r05/e_valu_rates3.txt)"},
                  open(a.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
