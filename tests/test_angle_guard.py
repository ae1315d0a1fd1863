"""Angle-list input guard: TemplateMatcher.cpp:130-144 accumulates `a += step` until the tolerance,
so a non-finite tolerance or step, or a step so small that the list would pass 100000 angles, would loop without end
or exhaust memory in the reference.  Engine and oracle both refuse such parameters with FPM_E_INVALID_ARG (no
search, no results).  (A NaN top_angle_step is not > 0, so it selects the reference's derived step, as 0 does.)"""
import math

import pytest

from fastest_image_pattern_matching_amd import _lib as L
from fastest_image_pattern_matching_amd import synth
from tests import oracle

BAD = [dict(tolerance_angle=math.nan), dict(tolerance_angle=math.inf), dict(tolerance_angle=180.0, top_angle_step=1e-9),
       dict(tolerance_angle=1e12)]


def _scene(templates):
    t = templates["Dst10"]
    s = synth.noise(240, 200, 128, 10, 3)
    synth.paste_rotated(s, t, 120, 100, 20.0)
    return s, t


@pytest.mark.parametrize("prm", BAD)
def test_oracle_refuses_unbounded_angle_lists(templates, prm):
    s, t = _scene(templates)
    o = oracle.OracleMatcher().set(**prm)
    assert o.learnPattern(t)
    rc, res = o.match_raw(s)
    assert rc == L.FPM_E_INVALID_ARG and res == []


@pytest.mark.gpu
@pytest.mark.parametrize("prm", BAD)
def test_engine_refuses_unbounded_angle_lists(gpu_matcher_factory, templates, prm):
    s, t = _scene(templates)
    m = gpu_matcher_factory(**prm)
    assert m.learnPattern(t)
    assert m.match(s) == []
    assert "angle list" in m.last_error()
