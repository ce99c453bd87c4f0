"""The MATLAB boundary: one MEX shim per reference function in
mex/, each shadowing the .m file of the same name.  MATLAB is absent, so the
shims are compiled -fsyntax-only against include/calanczos.h and a
declarations-only header of the documented MEX API (mex/syntax/mex.h): a
signature drift in the C ABI breaks this test.  CPU only."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MEX = os.path.join(ROOT, "mex")
# the reference files the shims shadow (SURVEY §8b's signatures to preserve)
SHADOWED = {"SpMV", "matrix_powers_monomial", "matrix_powers_newton", "tsqr", "cholqr", "normalize", "project",
            "projectAndNormalize", "ca_lanczos", "restarted_ca_lanczos", "impl_restarted_ca_lanczos"}


def test_every_hot_path_function_has_a_shim():
    shims = {f[: -len("_mex.c")] for f in os.listdir(MEX) if f.endswith("_mex.c")}
    assert shims == SHADOWED


def test_shims_compile_against_the_abi():
    p = subprocess.run(["make", "-C", MEX, "check"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "11 checked" in p.stdout


def test_shims_call_declared_entry_points():
    hdr = open(os.path.join(ROOT, "include", "calanczos.h")).read()
    declared = set(re.findall(r"\b(cal_[a-z0-9_]+)\s*\(", hdr))
    for f in sorted(os.listdir(MEX)):
        if f.endswith(".c") or f.endswith(".h"):
            src = open(os.path.join(MEX, f)).read()
            used = {u for u in re.findall(r"\b(cal_[a-z0-9_]+)\s*\(", src) if not u.startswith("cal_mex_")}
            assert used <= declared, (f, used - declared)
