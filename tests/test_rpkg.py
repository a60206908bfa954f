"""The R package skeleton (mkgpu/) stays consistent with include/mk.h.  R is not installed in
this image, so the glue is never compiled or run here; these checks catch drift between the
C-ABI, the .Call glue (mkgpu/src/mk_r.c) and the R wrappers (mkgpu/R/mkgpu.R) statically."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(*p):
    with open(os.path.join(ROOT, *p)) as f:
        return f.read()


def _struct_fields(header, name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), header, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"(\w+)\s*;", body)


def test_every_config_and_problem_field_is_set_by_the_glue():
    h, c = _read("include", "mk.h"), _read("mkgpu", "src", "mk_r.c")
    for f in _struct_fields(h, "mk_config"):
        assert re.search(r"\bc\.%s\s*=" % f, c), f"mk_r_fit leaves mk_config.{f} unset"
    for f in _struct_fields(h, "mk_problem"):
        assert re.search(r"\bpr\.%s\s*=" % f, c), f"mk_r_fit leaves mk_problem.{f} unset"


def test_call_registrations_match_c_signatures_and_r_calls():
    c, r = _read("mkgpu", "src", "mk_r.c"), _read("mkgpu", "R", "mkgpu.R")
    reg = dict((n, int(k)) for n, k in re.findall(r'\{"(\w+)", \(DL_FUNC\)&\w+, (\d+)\}', c))
    assert set(reg) == {"mk_r_fit", "mk_r_combine", "mk_r_summary", "mk_r_glm"}
    for name, nargs in reg.items():
        sig = re.search(r"SEXP %s\((.*?)\) \{" % name, c, re.S).group(1)
        assert sig.count("SEXP") == nargs, name
    # every .Call in the R code names a registered routine with that many arguments
    for m in re.finditer(r'\.Call\("(\w+)",', r):
        name = m.group(1)
        assert name in reg, name
        depth, i, args = 1, m.end(), 0
        while depth:
            ch = r[i]
            if ch in "([":
                depth += 1
            elif ch in ")]":
                depth -= 1
            elif ch == "," and depth == 1:
                args += 1
            i += 1
        assert args + 1 == reg[name], (name, args + 1, reg[name])


def test_glue_calls_only_declared_entry_points():
    h, c = _read("include", "mk.h"), _read("mkgpu", "src", "mk_r.c")
    declared = set(re.findall(r"\b(mk_\w+)\s*\(", h))
    used = set(re.findall(r"\b(mk_(?!r_)\w+)\s*\(", c))
    assert used <= declared, used - declared
    # the config list the R wrapper builds has one entry per cfg index the glue reads
    n_cfg = max(int(i) for i in re.findall(r"VECTOR_ELT\(cfg, (\d+)\)", c)) + 1
    r = _read("mkgpu", "R", "mkgpu.R")
    body = r[r.index("cfg <- list("):]
    depth, i, items = 0, body.index("(") , 1
    while True:
        ch = body[i]
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
            if depth == 0:
                break
        elif ch == "," and depth == 1:
            items += 1
        i += 1
    assert items == n_cfg, (items, n_cfg)
