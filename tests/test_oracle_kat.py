"""The oracle (oracle/rtc_oracle.hpp) against the reference's own unit-test
known answers (tests/golden/reference_kats.json, transcribed with file:line).
This is what pins the oracle before any GPU result is compared with it."""
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ORACLE

EPSILON = 8e-8  # consts.rs:2 (coarse_eq, utils.rs:16-24)


@pytest.fixture(scope="module")
def computed():
    exe = os.path.join(ORACLE, "_build", "kat_runner")
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return json.loads(out)


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)["cases"]


def test_every_golden_case_is_computed(computed, golden):
    assert set(golden) <= set(computed)


@pytest.mark.parametrize("name", sorted(json.load(open(os.path.join(GOLDEN, "reference_kats.json")))["cases"]))
def test_known_answer(name, computed, golden):
    case = golden[name]
    got, exp, mode = computed[name], case["expected"], case["mode"]
    if mode == "terminates":
        return
    if mode == "predicate":
        if name == "intersection.hit_offsets_point":  # intersection.rs:160-171
            over_z, z = got
            assert over_z < -EPSILON / 2 and z > over_z
        elif name == "intersection.under_point_below_surface":  # intersection.rs:240-253
            under_z, z = got
            assert under_z > EPSILON / 2 and z < under_z
        else:
            pytest.fail(f"no predicate for {name}")
        return
    assert len(got) == len(exp), (got, exp)
    for g, e in zip(got, exp):
        if mode == "exact":
            assert g == e, f"{name} ({case['src']}): {got} != {exp}"
        else:
            assert g == e or abs(g - e) < EPSILON, f"{name} ({case['src']}): {got} vs {exp}"
