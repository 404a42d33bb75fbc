"""CPU: param_factory::make_ssd_params and batch_sampler::sample_patches (aeon
src/augment_image.cpp:232-586) -- the product's C ABI against aeon's own known-answer tests
(test/test_augmentation.cpp:246-443) and against the oracle's independent restatement."""
import math

import numpy as np
import pytest

import aeon_amd as A
from tests import helpers as H

ALL_CONSTRAINTS = {"min_jaccard_overlap": 0.2, "max_jaccard_overlap": 0.3, "min_sample_coverage": 0.4,
                   "max_sample_coverage": 0.5, "min_object_coverage": 0.6, "max_object_coverage": 0.7}
OBJECTS = [(0, 0, 1, 1), (0, 0, 0.5, 0.5)]


def _both(aug):
    return A.ParamFactory(aug), H.O.Factory(H.oracle_aug_config(aug))


def test_make_ssd_params_default(oracle):
    """image_augmentation.make_ssd_params_default (test_augmentation.cpp:246-274)."""
    aug = {"type": "image", "crop_enable": False}
    for f, make in ((A.ParamFactory(aug).make_ssd_params, None),
                    (None, oracle.make_ssd_params)):
        st = np.array([1], np.uint32)
        p = f(st, 100, 100, 200, 300) if f else make(oracle.Factory(H.oracle_aug_config(aug)), st, 100, 100, 200, 300)
        assert (p.crop_x, p.crop_y, p.crop_w, p.crop_h) == (0, 0, 100, 100)
        assert (p.expand_x, p.expand_y, p.expand_w, p.expand_h) == (0, 0, 100, 100)
        assert p.expand_ratio == 1.0
        assert (p.flip, p.angle, p.hue, p.n_lighting, p.color_noise_std) == (0, 0, 0, 0, 0)
        assert (p.contrast, p.brightness, p.saturation) == (1.0, 1.0, 1.0)
        assert (p.out_w, p.out_h) == (200, 300)


def test_make_ssd_params_transformations(oracle):
    """image_augmentation.make_ssd_params_transformations (test_augmentation.cpp:276-317)."""
    aug = {"type": "image", "crop_enable": False, "expand_ratio": [4.0, 4.0], "expand_probability": 1.0,
           "batch_samplers": [{"max_sample": 1, "max_trials": 50,
                               "sampler": {"scale": [0.5, 0.5], "aspect_ratio": [1.0, 1.0]}}]}
    f, of = _both(aug)
    for seed in range(1, 40):
        s1, s2 = np.array([seed], np.uint32), np.array([seed], np.uint32)
        p = f.make_ssd_params(s1, 10, 10, 20, 30, [(0, 0, 1, 1)])
        q = oracle.make_ssd_params(of, s2, 10, 10, 20, 30, [(0, 0, 1, 1)])
        for r in (p, q):
            assert (r.crop_w, r.crop_h) == (20, 20)
            assert r.expand_x <= 30 and r.expand_y <= 30
            assert (r.expand_w, r.expand_h) == (40, 40)
            assert r.expand_ratio == 4.0
            assert (r.out_w, r.out_h) == (20, 30)
            assert (r.flip, r.angle, r.hue) == (0, 0, 0)
        assert p.as_dict() == q.as_dict() and s1[0] == s2[0]


def test_max_sample(oracle):
    """image_augmentation.max_sample (test_augmentation.cpp:347-376): the whole-image sample
    passes the constraints through `found` carrying over from the second object
    (augment_image.cpp:410-461), so exactly max_sample samples are kept."""
    aug = {"type": "image", "crop_enable": False,
           "batch_samplers": [{"max_sample": 10, "max_trials": 50,
                               "sampler": {"scale": [1, 1], "aspect_ratio": [1, 1]},
                               "sample_constraint": ALL_CONSTRAINTS}, {}]}
    f, of = _both(aug)
    s1, s2 = np.array([5], np.uint32), np.array([5], np.uint32)
    assert len(f.sample_patches(0, s1, OBJECTS)) == 10
    assert len(oracle.sample_patches(of, 0, s2, OBJECTS)) == 10
    assert s1[0] == s2[0]


def test_max_trials(oracle):
    """image_augmentation.max_trials (test_augmentation.cpp:378-411)."""
    rng = np.random.default_rng(0)
    for _ in range(10):
        max_trials = int(1 + rng.integers(0, 100))
        aug = {"type": "image", "crop_enable": False,
               "batch_samplers": [{"max_sample": 1000, "max_trials": max_trials,
                                   "sampler": {"scale": [1, 1], "aspect_ratio": [1, 1]},
                                   "sample_constraint": ALL_CONSTRAINTS}, {}]}
        f, of = _both(aug)
        s1, s2 = np.array([9], np.uint32), np.array([9], np.uint32)
        a = f.sample_patches(0, s1, OBJECTS)
        b = oracle.sample_patches(of, 0, s2, OBJECTS)
        assert len(a) <= max_trials and a == b and s1[0] == s2[0]


def test_default_patch(oracle):
    """image_augmentation.default_patch (test_augmentation.cpp:413-443): every sample that
    satisfies these point constraints is the whole image."""
    aug = {"type": "image", "crop_enable": False,
           "batch_samplers": [{"max_sample": 10, "max_trials": 50,
                               "sampler": {"scale": [0.1, 1], "aspect_ratio": [0.5, 2]},
                               "sample_constraint": {"min_jaccard_overlap": 0.3, "max_jaccard_overlap": 0.3,
                                                     "min_sample_coverage": 0.4, "max_sample_coverage": 0.4,
                                                     "min_object_coverage": 0.5, "max_object_coverage": 0.5}}]}
    f, of = _both(aug)
    for seed in (1, 2, 3, 77):
        s1, s2 = np.array([seed], np.uint32), np.array([seed], np.uint32)
        a = f.sample_patches(0, s1, OBJECTS)
        assert a == oracle.sample_patches(of, 0, s2, OBJECTS)
        for b in a:
            assert all(abs(x - y) < 1e-5 for x, y in zip(b, (0, 0, 1, 1)))


SAMPLER_OBJECTS = [(0.2, 0.2, 0.6, 0.4), (0, 0, 0.4, 0.4), (0.5, 0.5, 0.6, 0.6), (0.2, 0.2, 0.8, 0.6),
                   (0.1, 0.0, 0.9, 1.0), (0.0, 0.1, 1.0, 0.9), (0, 0, 1, 1), (0, 0, 1, 1),
                   (0.345, 0.345, 0.35, 0.35), (0.9, 0.9, 0.91, 0.91), (0.1, 0.9, 0.15, 0.95),
                   (0.9, 0.1, 0.95, 0.15), (0.56, 0.17, 0.41 + 0.56, 0.17 + 0.59)]


def _check_sampler(oracle, aspect, scale, what="min_jaccard_overlap", mv=0.1):
    """test_sampler (test_augmentation.cpp:30-78): 50 draws from a max_sample 1 sampler; every
    sample lies in [0, 1] and keeps the configured aspect ratio (width / height)."""
    aug = {"type": "image", "crop_enable": False,
           "batch_samplers": [{"max_sample": 1, "max_trials": 50,
                               "sampler": {"scale": [scale, scale], "aspect_ratio": [aspect, aspect]},
                               "sample_constraint": {what: mv}}]}
    f, of = _both(aug)
    s1, s2 = np.array([17], np.uint32), np.array([17], np.uint32)
    non_full = 0
    for _ in range(50):
        a = f.sample_patches(0, s1, SAMPLER_OBJECTS)
        assert a == oracle.sample_patches(of, 0, s2, SAMPLER_OBJECTS) and s1[0] == s2[0]
        for x0, y0, x1, y1 in a:
            assert x0 >= 0 and y0 >= 0 and x1 <= 1 and y1 <= 1
            if (x0, y0, x1, y1) != (0, 0, 1, 1):
                assert math.isclose((x1 - x0) / (y1 - y0), aspect, rel_tol=4e-7 * 4)
                assert x1 - x0 > 0
                non_full += 1
    if not (aspect == 1 and scale == 1):
        assert non_full > 0


@pytest.mark.parametrize("aspect,scale", [(1, 0.5), (1, 1), (2, 0.5), (2, 0.2), (0.4, 0.6)])
def test_batch_sampler_ratio_scale(oracle, aspect, scale):
    """image_augmentation.batch_sampler_ratio_scale (test_augmentation.cpp:319-326)."""
    _check_sampler(oracle, aspect, scale)


def test_batch_sampler_random_sample_constraint(oracle):
    """image_augmentation.batch_sampler_random_sample_constraint (test_augmentation.cpp:328-345),
    seeded here instead of std::random_device."""
    rng = np.random.default_rng(12)
    kinds = ["_jaccard_overlap", "_sample_coverage", "_object_coverage"]
    for i in range(20):
        v1 = float(np.float32(rng.random()))
        _check_sampler(oracle, 0.7, 0.5, ("max" if v1 > 0.9 else "min") + kinds[i % 3], v1)


SSD_AUG = {"type": "image", "crop_enable": False, "flip_enable": True, "expand_ratio": [1.0, 4.0],
           "expand_probability": 0.5, "brightness": [0.875, 1.125], "saturation": [0.5, 1.5],
           "batch_samplers": [
               {"max_sample": 1, "max_trials": 50,
                "sampler": {"scale": [0.3, 1.0], "aspect_ratio": [0.5, 2.0]},
                "sample_constraint": {"min_jaccard_overlap": 0.1}},
               {"max_sample": 1, "max_trials": 50,
                "sampler": {"scale": [0.3, 1.0], "aspect_ratio": [0.5, 2.0]},
                "sample_constraint": {"min_object_coverage": 0.5, "max_sample_coverage": 0.9}},
               {"max_trials": 1}]}


def random_boxes(rng, w, h, n):
    res = []
    for _ in range(n):
        x0, y0 = float(rng.integers(0, w - 1)), float(rng.integers(0, h - 1))
        res.append((x0, y0, float(rng.integers(int(x0), w)), float(rng.integers(int(y0), h))))
    return res


def test_make_ssd_params_matches_oracle(oracle):
    """Random SSD configurations: product params and engine state equal the oracle's."""
    f, of = _both(SSD_AUG)
    rng = np.random.default_rng(4)
    states = A.seed_slots(11, 32)
    for i in range(32):
        s1, s2 = states[i:i + 1].copy(), states[i:i + 1].copy()
        for _ in range(4):
            w, h = int(rng.integers(20, 700)), int(rng.integers(20, 700))
            boxes = random_boxes(rng, w, h, int(rng.integers(0, 5)))
            p = f.make_ssd_params(s1, w, h, 300, 300, boxes)
            q = oracle.make_ssd_params(of, s2, w, h, 300, 300, boxes)
            assert p.as_dict() == q.as_dict(), (p.as_dict(), q.as_dict())
            assert s1[0] == s2[0]
            assert 0 <= p.crop_x and p.crop_x + p.crop_w <= p.expand_w + 1
            assert 0 <= p.crop_y and p.crop_y + p.crop_h <= p.expand_h + 1


def test_ssd_errors():
    f = A.ParamFactory({"type": "image", "crop_enable": False, "expand_ratio": [4.0, 4.0],
                        "expand_probability": 1.0})
    st = np.array([1], np.uint32)
    with pytest.raises(A.AeonHipError):  # boundingbox::expand refuses a box outside the canvas
        f.make_ssd_params(st, 10, 10, 20, 20, [(0, 0, 45, 5)])
    with pytest.raises(A.AeonHipError):
        f.sample_patches(3, st, [])
