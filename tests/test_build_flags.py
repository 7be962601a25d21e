"""The device code's exactness rests on compile flags that leave no macro to
test from inside the source: no contraction, no fast
math, correctly rounded f32 division / sqrt, and no SLP vectorisation (the
ROCm 7.2 backend miscompiles the vectorised triangle test of the any-hit walk;
profiles/r03_slp/).  Every build recipe of device code that must be exact has
to carry all four; ptg_device_selftest() checks the contraction at run time."""
import os
import re

from conftest import ROOT

PKG = os.path.join(ROOT, "path-tracing...but-on-the-lumi-cluster_amd")
REQUIRED = ("-ffp-contract=off", "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize")
RECIPES = [os.path.join(PKG, "csrc", "Makefile"), os.path.join(ROOT, "tests", "device_dropin", "Makefile"),
           os.path.join(ROOT, "tools", "exhaustive_f64.sh")]


def test_exact_build_recipes_carry_the_flags():
    for path in RECIPES:
        text = open(path).read()
        missing = [f for f in REQUIRED if f not in text]
        assert not missing, "%s lacks %s" % (os.path.relpath(path, ROOT), missing)


def test_device_header_documents_the_flags():
    text = open(os.path.join(ROOT, "include", "ptg_device.h")).read()
    for f in REQUIRED:
        assert f in text, f
    assert re.search(r"#if defined\(__FAST_MATH__\)\s*\n#error", text)
    assert "ptg_device_selftest" in text
