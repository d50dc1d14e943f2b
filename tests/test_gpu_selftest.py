"""The kernels' exact-reciprocal fast sequence (prt_device.h rcp_fast_seq), swept over all 2^32 floats
on the GPU against the IEEE division 1.0f / b (prt_selftest_rcp): rcp_exact takes it only for
|b| in [2^-40, 2^40], where it must equal the division bit for bit — the Moller-Trumbore test's
1 / det (intersection_taichi.py:69-91) and with it every image rests on that."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CLASSES = ("zero", "denormal", "normal < 2^-40", "[2^-40, 2^40]", "(2^40, 2^126]", "> 2^126", "inf", "nan")


def test_fast_reciprocal_is_the_ieee_division_where_the_kernels_use_it():
    from pyrenderer_amd import _native as N
    mism = np.zeros(8, np.uint64)
    N.check(N.lib().prt_selftest_rcp(0, N.ptr(mism)))
    report = dict(zip(CLASSES, mism.tolist()))
    print("fast reciprocal mismatches by class:", report)
    assert report["[2^-40, 2^40]"] == 0, report
    # measured on gfx950: exact for every normal |b| <= 2^126, not for zero / denormal / huge / infinite
    # operands (rcp_exact sends those to the division; a zero det is masked by det != 0 anyway)
    assert report["normal < 2^-40"] == 0 and report["(2^40, 2^126]"] == 0, report
