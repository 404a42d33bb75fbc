"""CPU: the product's host param_factory (aeon_amd C ABI) against the oracle's restatement of
aeon's make_params (src/augment_image.cpp:107-230) and config validation."""
import json

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

AUGS = {
    "C1": C.C1_AUG, "C2": C.C2_AUG, "C3": C.C3_AUG, "C5": C.C5_AUG,
    "area": {"type": "image", "do_area_scale": True, "scale": [0.08, 1.0],
             "horizontal_distortion": [0.75, 1.33], "flip_enable": True, "center": False},
    "hdist": {"type": "image", "scale": [0.3, 0.9], "horizontal_distortion": [0.5, 2.0], "center": False,
              "angle": [0, 0], "lighting": [0.0, 0.5]},
    "nocrop_pad": {"type": "image", "crop_enable": False, "padding": 4, "flip_enable": True},
    "nocrop_fixed": {"type": "image", "crop_enable": False, "fixed_scaling_factor": 0.5},
}


@pytest.mark.parametrize("name", sorted(AUGS))
def test_make_params_matches_oracle(oracle, name):
    aug = AUGS[name]
    f = A.ParamFactory(aug)
    of = oracle.Factory(H.oracle_aug_config(aug))
    states = A.seed_slots(7, 16)
    assert np.array_equal(states, oracle.seed_slots(7, 16))
    rng = np.random.default_rng(1)
    for i in range(16):
        s1, s2 = states[i:i + 1].copy(), states[i:i + 1].copy()
        for _ in range(4):  # the slot engine persists across decode windows
            w, h = int(rng.integers(16, 900)), int(rng.integers(16, 900))
            p = f.make_params(s1, w, h, 224, 224)
            q = of.make_params(s2, w, h, 224, 224)
            assert p.as_dict() == q.as_dict(), (name, p.as_dict(), q.as_dict())
            assert s1[0] == s2[0]


def test_seed_slots_is_minstd():
    # minstd_rand0(1): 16807, 282475249, ... (the C++11 reference values)
    assert list(A.seed_slots(1, 3)) == [16807, 282475249, 1622650073]


@pytest.mark.parametrize("bad", [
    {"type": "image", "scale": [0.5, 1.5]},
    {"type": "image", "scale": [0.9, 0.5]},
    {"type": "image", "angle": [10, -10]},
    {"type": "image", "contrast": [1.0, 0.5]},
    {"type": "image", "hue": [5, -5]},
    {"type": "image", "expand_ratio": [0.5, 2.0]},
    {"type": "image", "batch_samplers": [{}], "crop_enable": True},
    {"scale": [0.5, 1.0]},
])
def test_invalid_configs(bad):
    with pytest.raises(A.AeonHipError) as e:
        A.ParamFactory(bad)
    assert e.value.code == A.AEON_HIP_EINVAL


def test_padding_with_crop_enable_throws():
    f = A.ParamFactory({"type": "image", "padding": 4})
    with pytest.raises(A.AeonHipError):
        f.make_params(np.array([1], np.uint32), 32, 32, 32, 32)


def test_unknown_interpolation_fails_per_record():
    # aeon resolves the method when a record is resized (image.cpp:38-50), not at config time
    f = A.ParamFactory({"type": "image", "interpolation_method": "BICUBICAL"})
    with pytest.raises(A.AeonHipError):
        f.make_params(np.array([1], np.uint32), 32, 32, 32, 32)


def test_bad_json():
    with pytest.raises(A.AeonHipError):
        A.ParamFactory("{not json")
    # aeon does not verify unknown augmentation keys (augment_image.cpp:50)
    A.ParamFactory(json.dumps({"type": "image", "some_future_key": 1}))


def test_fixed_aspect_ratio_output_sizes():
    """image.var_resize_fixed_ratio / var_resize_fixed_scale (test/test_image.cpp:1070-1130):
    crop_enable=false scales the whole record to fit the 400x400 canvas (300x200 -> 400x267),
    or by fixed_scaling_factor (1.0 -> 300x200)."""
    for extra, want in (({}, (400, 267)), ({"fixed_scaling_factor": 1.0}, (300, 200))):
        aug = dict({"type": "image", "fixed_aspect_ratio": True, "crop_enable": False}, **extra)
        (p,) = H.draw_params(aug, [(300, 200)], 400, 400)
        assert (p.out_w, p.out_h) == want
        assert (p.crop_x, p.crop_y, p.crop_w, p.crop_h) == (0, 0, 300, 200)
