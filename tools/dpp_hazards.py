"""Check the hand-placed wait states of the fused-DPP fmacs (mk_linalg.hip `fmac_bc16`).

A DPP read of a VGPR needs two wait states after a VALU write of it (gfx9 family).  The fused
v_fmac_f64_dpp is inline asm, which the compiler's hazard recognizer does not look inside, so the
callers put an `s_nop 1` where their program order needs one.  This walks the compiled ISA and
flags any v_fmac_f64_dpp whose DPP source was written by a VALU instruction fewer than two wait
states earlier (s_nop N counts N + 1; other instructions count one each; conservatively only VALU
and s_nop are counted).  Usage: python tools/dpp_hazards.py file.s  (exit 1 on a hazard)."""
import re
import sys


def _regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


def check(text):
    ins = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith((";", ".")) or line.endswith(":"):
            # a label or directive starts a new block: be conservative and keep walking (branches
            # into the middle of a DPP sequence do not occur in these kernels)
            continue
        ins.append(line)
    n, bad = 0, []
    for i, line in enumerate(ins):
        if not line.startswith("v_fmac_f64_dpp"):
            continue
        n += 1
        ops = [o.strip() for o in line.split(None, 1)[1].split(",")]
        src = _regs(ops[1].split()[0])
        ws, j = 0, i - 1
        while j >= 0 and ws < 2:
            p = ins[j]
            if p.startswith("s_nop"):
                ws += int(p.split()[1]) + 1
            elif p.startswith("v_"):
                parts = p.split(None, 1)
                dst = _regs(parts[1].split(",")[0].strip()) if len(parts) > 1 else set()
                if dst & src:
                    bad.append((p, line))
                    break
                ws += 1
            j -= 1
    return n, bad


if __name__ == "__main__":
    n, bad = check(open(sys.argv[1]).read())
    for p, line in bad:
        print("HAZARD:", p, "->", line)
    print(f"{n} fused DPP fmacs, {len(bad)} hazards")
    sys.exit(1 if bad else 0)
