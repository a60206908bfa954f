"""The R package skeleton (mkgpu/) stays consistent with include/mk.h.  R is not installed in
this image, so the glue is never linked or run here; these checks catch drift between the
C-ABI, the .Call glue (mkgpu/src/mk_r.c) and the R wrappers (mkgpu/R/mkgpu.R) statically, and
type-check the glue against mk.h with gcc over stub declarations of the R API (tests/rstub/)."""
import os
import re
import shutil
import subprocess

import pytest

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
        assert re.search(r"\bc->%s\s*=" % f, c), f"read_config leaves mk_config.{f} unset"
    for f in _struct_fields(h, "mk_problem"):
        assert re.search(r"\bpr->%s\s*=" % f, c), f"read_problem leaves mk_problem.{f} unset"
    for f in _struct_fields(h, "mk_combined"):
        if f not in ("exchange", "comm_ranks"):    # outputs
            assert re.search(r"\bcb\.%s\s*=" % f, c), f"mk_r_fit leaves mk_combined.{f} unset"


def test_call_registrations_match_c_signatures_and_r_calls():
    c, r = _read("mkgpu", "src", "mk_r.c"), _read("mkgpu", "R", "mkgpu.R")
    reg = dict((n, int(k)) for n, k in re.findall(r'\{"(\w+)", \(DL_FUNC\)&\w+, (\d+)\}', c))
    assert set(reg) == {"mk_r_fit", "mk_r_spmvglm", "mk_r_sppredict", "mk_r_combine", "mk_r_summary", "mk_r_glm",
                        "mk_r_hw_queues", "mk_r_hip_started", "mk_r_shutdown"}
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


def test_r_wrappers_mirror_the_reference_calls():
    """mk_spMvGLM / mk_spPredict take spBayes's argument names as MK.R:80-87 passes them, the
    fit runs batch by batch with the interrupt check, coordinates are coerced with as.matrix,
    and mk_meta_fit hands its device list to the multi-device entry point."""
    r, c = _read("mkgpu", "R", "mkgpu.R"), _read("mkgpu", "src", "mk_r.c")
    sig = re.search(r"mk_spMvGLM <- function\((.*?)\) \{", r, re.S).group(1)
    for arg in ("formula", "coords", "weights", "starting", "tuning", "priors", "amcmc", "cov.model", "n.report"):
        assert re.search(r"\b%s\b" % re.escape(arg), sig), arg
    sig = re.search(r"mk_spPredict <- function\((.*?)\) \{", r, re.S).group(1)
    for arg in ("sp.obj", "pred.coords", "pred.covars", "start", "end"):
        assert re.search(r"\b%s\b" % re.escape(arg), sig), arg
    for field in ("p.beta.theta.samples", "p.w.samples", "p.w.predictive.samples"):
        assert field in r
    assert "devices = 0L" in r and "as.integer(devices)" in r
    assert "R_ToplevelExec(check_interrupt" in c and "R_CheckUserInterrupt()" in c
    assert "mk_meta_fit(&pr, &c, INTEGER(devices)" in c
    assert c.count("mk_session_run(") == 1 and "for (int it = 0; it < n_samples; it += c.batch_length)" in c
    assert r.count(".mk_coords(") >= 4          # coords, coords.test, pred.coords coerced
    exports = re.search(r"export\((.*?)\)", _read("mkgpu", "NAMESPACE"), re.S).group(1)
    for fn in ("mk_meta_fit", "mk_spMvGLM", "mk_spPredict", "mk_combine", "mk_posterior_summary"):
        assert fn in exports


def test_onload_passes_the_queue_count_hip_started_with():
    """.onLoad raises GPU_MAX_HW_QUEUES only while HIP has not started (libmk then reads the variable
    itself: mk_set_hw_queues(-1)); when another package started HIP first it reports the count HIP
    started with (the variable as it was, else HIP's default 4), never a blanket 8.
    The pooled streams are released at unload and at R's exit."""
    r, c = _read("mkgpu", "R", "mkgpu.R"), _read("mkgpu", "src", "mk_r.c")
    body = r[r.index(".onLoad <- function"):]
    body = body[:body.index("\n}\n") + 3]
    assert 'if (.Call("mk_r_hip_started"))' in body
    started, fresh = body.split("} else {")
    assert '.Call("mk_r_hw_queues", if (q > 0L) q else 4L)' in started
    assert "Sys.setenv" not in started
    assert 'Sys.setenv(GPU_MAX_HW_QUEUES = "8")' in fresh and '.Call("mk_r_hw_queues", -1L)' in fresh
    assert 'reg.finalizer(.mk_exit, function(e) .Call("mk_r_shutdown"), onexit = TRUE)' in body
    assert '.Call("mk_r_shutdown")' in r[r.index(".onUnload"):]
    assert "mk_hip_initialized()" in c and "mk_shutdown();" in c


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not on PATH")
def test_glue_type_checks_against_the_c_abi():
    """gcc -fsyntax-only over mk_r.c with tests/rstub/ standing in for R's headers (declarations of
    the R entry points the glue uses, with R's signatures): every mk_* call, struct field and
    pointer type the glue hands to include/mk.h is checked by the compiler.  Linking against R
    and running under R stay untested (no R in the image)."""
    cmd = ["gcc", "-fsyntax-only", "-std=c99", "-Wall", "-Werror=implicit-function-declaration",
           "-Werror=incompatible-pointer-types", "-Werror=int-conversion", "-Werror=return-type",
           "-I", os.path.join(ROOT, "tests", "rstub"), "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "mkgpu", "src", "mk_r.c")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "warning" not in r.stderr, r.stderr
