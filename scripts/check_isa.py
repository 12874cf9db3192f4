"""Static checks of the gfx950 machine code of the block codec (CPU-only; tests/test_isa.py runs it).

1. SCC across the compare-exchange strings.  The sort networks' inline asm (bra_hip_common.h cx*)
   computes its lane mask with `s_xnor_b64` / `s_xor_b64 vcc, vcc, ...`, which also write SCC.  If the compiler
   believes SCC survives the string (a missing "scc" clobber), a later s_cselect / s_cbranch_scc
   reads the xnor's result instead of the compiler's own compare: a network stage silently takes
   the wrong direction for some key sets.  Flagged: an SCC reader whose nearest preceding SCC writer
   (same straight-line code) is such an xnor.
2. VALU write -> DPP / v_permlane*_swap read with fewer than 2 wait states (the gfx950 rule hipcc
   pads for its own instructions but not around inline asm).

Input: the product objects (br-archive_amd/build/*.o: the gfx950 code object is unbundled from
.hip_fatbin and disassembled) or assembly files (hipcc -S --cuda-device-only).

    python scripts/check_isa.py [files...]       exit 1 on a finding
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/llvm/bin"
SCC_READ = re.compile(r"^(s_cselect_|s_cbranch_scc[01]|s_cmov_|s_cmovk_|s_addc_|s_subb_)")
SCC_WRITE = re.compile(
    r"^(s_cmp|s_bitcmp|s_add_|s_sub_|s_addc_|s_subb_|s_and_|s_or_|s_xor_|s_xnor_|s_nand_|s_nor_|s_andn2_|s_orn2_|s_not_|"
    r"s_lshl|s_lshr|s_ashr|s_bfe_|s_bcnt|s_min_|s_max_|s_abs|s_absdiff|s_cmpk_|s_quadmask|s_wqm)")
BLOCK_END = re.compile(r"^(s_branch|s_cbranch|s_setpc|s_endpgm|s_swappc)")
DPP = re.compile(r"_dpp\b|\bquad_perm:|\brow_(shl|shr|ror|mirror|half_mirror|bcast|newbcast|share|xmask)|\bwave_(shl|shr|rol|ror)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _regs(text: str):
    out = []
    for m in VREG.finditer(text):
        out.extend([int(m.group(3))] if m.group(3) is not None else range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def instructions(path: str):
    """(function, instruction text) pairs of an assembly file or of a built object's gfx950 code."""
    if path.endswith(".o"):
        with tempfile.TemporaryDirectory() as td:
            fb, co = os.path.join(td, "fb"), os.path.join(td, "co")
            subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb], check=True)
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--input={fb}", f"--output={co}", "--unbundle"], check=True)
            text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout
        fn = "?"
        for line in text.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                fn = m.group(1)
                yield fn, ":"
                continue
            t = line.split("//")[0].strip()
            if t and not t.endswith(":"):
                yield fn, t
        return
    fn = "?"
    with open(path) as f:
        for line in f:
            t = line.strip()
            if not t or t.startswith(";") or t.startswith("."):
                continue
            if t.endswith(":"):
                if not t.startswith(".L"):
                    fn = t[:-1]
                yield fn, ":"  # a branch target: straight-line code ends
                continue
            yield fn, t.split(";")[0].strip()


def check(path: str):
    findings = []
    recent = []  # (instruction) of the current straight-line region, newest last
    last_write = {}
    t = 0
    for fn, ins in instructions(path):
        if ins == ":":
            recent.clear()
            continue
        op = ins.split(None, 1)[0]
        args = ins.split(None, 1)[1] if " " in ins else ""
        # 1. SCC reader fed by an asm xnor
        if SCC_READ.match(op):
            for prev in reversed(recent):
                if SCC_WRITE.match(prev.split(None, 1)[0]):
                    if re.match(r"s_xn?or_b64 vcc, vcc", prev):
                        findings.append(f"{os.path.basename(path)} [{fn}] `{ins}` reads SCC written by `{prev}` (inline asm without an scc clobber)")
                    break
        # 2. VALU write -> DPP / permlane swap read
        if op == "s_nop":
            t += int(args.strip() or "0", 0) + 1
            recent.append(ins)
            continue
        if op.startswith("v_") and (DPP.search(ins) or op.startswith("v_permlane")):
            ops = [a.strip() for a in args.split(",")]
            if op.startswith("v_permlane"):
                srcs = _regs(ops[0]) + (_regs(ops[1]) if len(ops) > 1 else [])
            else:
                # sources; the destination too when its old value can be kept (a partial row / bank
                # mask, or a shift without bound_ctrl that leaves lanes without a source)
                partial = "row_mask:0xf" not in ins or "bank_mask:0xf" not in ins or (
                    re.search(r"\brow_(shl|shr)|\bwave_", ins) and "bound_ctrl" not in ins)
                srcs = [r for a in (ops if partial else ops[1:]) for r in _regs(a.split()[0] if a else "")]
            for r in srcs:
                if r in last_write and t - last_write[r] < 2:
                    findings.append(f"{os.path.basename(path)} [{fn}] `{ins}` reads v{r} {t - last_write[r]} wait state(s) after a VALU write")
                    break
        t += 1
        if op.startswith("v_") and not op.startswith(("v_readlane", "v_readfirstlane", "v_cmp", "v_nop")) and args:
            for r in _regs(args.split(",")[0]):
                last_write[r] = t
        recent.append(ins)
        if BLOCK_END.match(op):
            recent.clear()
        elif len(recent) > 64:
            del recent[0]
    return findings


def main(argv):
    files = argv or sorted(glob.glob(os.path.join(ROOT, "br-archive_amd", "build", "*.o")))
    bad = []
    for p in files:
        bad += check(p)
    for b in bad[:40]:
        print(b)
    print(f"{len(files)} file(s), {len(bad)} finding(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
