"""Check the DPP read wait states around the inline-asm fused fmacs (mk_linalg.hip `fmac_bc16`).

A DPP read of a VGPR needs two wait states after a VALU write of it (gfx9 family).  The fused
v_fmac_f64_dpp is inline asm: the compiler's hazard recognizer neither looks inside it nor counts
it as a VALU write, so two kinds of hazard are invisible to the compiler:
  * an inline-asm fmac whose DPP source was written by any VALU instruction too recently (the
    callers place an `s_nop 1` where their program order needs one);
  * any DPP instruction -- compiler-emitted ones included (v_mov_b32_dpp of dpp_f64 / wave_sum_dpp)
    -- whose DPP source was written by an inline-asm fmac too recently (the compiler does not know
    the fmac wrote it, so it inserts no s_nop).
This walks the compiled ISA backwards from every DPP instruction (s_nop N counts N + 1 wait
states, every other instruction one; conservatively only VALU and s_nop are counted).  A label or
branch met before two wait states is an unknown predecessor: for an inline-asm fmac it is reported
(the walk cannot prove the block's entry safe); for a compiler DPP the compiler guards its own
cross-block writers, and inline-asm writers at the end of a predecessor block are caught from that
block's side only when they feed a DPP in it, so those are reported too.
Usage: python tools/dpp_hazards.py file.s  (exit 1 on a hazard)."""
import re
import sys

FUSED = "v_fmac_f64_dpp"


def _regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


def _is_dpp(line):
    return re.match(r"v_\w+_dpp\b", line) is not None


def _operands(line):
    parts = line.split(None, 1)
    return [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []


def check(text):
    """Returns (fused fmacs seen, DPP instructions checked, hazards [(writer, reader)])."""
    ins = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith((";", ".")):
            continue
        if line.endswith(":"):
            ins.append("LABEL " + line)
            continue
        ins.append(line)
    n_fused, n_dpp, bad = 0, 0, []
    for i, line in enumerate(ins):
        if not _is_dpp(line):
            continue
        n_dpp += 1
        fused = line.startswith(FUSED)
        n_fused += fused
        ops = _operands(line)
        if len(ops) < 2:
            continue
        src = _regs(ops[1].split()[0])
        ws, j = 0, i - 1
        while j >= 0 and ws < 2:
            p = ins[j]
            if p.startswith("LABEL") or p.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
                if fused or any(FUSED in q for q in ins[max(0, j - 2):j]):
                    bad.append((p + " (unknown predecessor)", line))
                break
            if p.startswith("s_nop"):
                ws += int(p.split()[1]) + 1
            elif p.startswith("v_"):
                pops = _operands(p)
                dst = _regs(pops[0]) if pops else set()
                if dst & src:
                    if fused or p.startswith(FUSED):
                        bad.append((p, line))
                    break   # a compiler-visible writer feeding a compiler DPP: the compiler's own s_nop rules
                ws += 1
            j -= 1
    return n_fused, n_dpp, bad


if __name__ == "__main__":
    n, n_dpp, bad = check(open(sys.argv[1]).read())
    for p, line in bad:
        print("HAZARD:", p, "->", line)
    print(f"{n} fused DPP fmacs, {n_dpp} DPP instructions checked, {len(bad)} hazards")
    sys.exit(1 if bad else 0)
