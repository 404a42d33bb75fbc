"""CPU: the C ABI library loads, exports every symbol include/aeon_hip.h declares, and its
struct layouts match the header (checked by a C probe compiled against the header)."""
import ctypes
import os
import subprocess
import tempfile

import aeon_amd as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    lib = A.lib()
    names = A.exported_symbols()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n


def test_struct_layout_matches_header():
    probe = r'''
#include <stdio.h>
#include <stddef.h>
#include "aeon_hip.h"
int main(void) {
  printf("%zu %zu %zu\n", sizeof(aeon_img_desc), sizeof(aeon_aug_params), sizeof(aeon_out_desc));
  printf("%zu %zu %zu\n", offsetof(aeon_aug_params, lighting), offsetof(aeon_aug_params, interp),
         offsetof(aeon_out_desc, item_stride));
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "p.c")
        open(src, "w").write(probe)
        exe = os.path.join(d, "p")
        subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), src, "-o", exe])
        a, b = subprocess.check_output([exe]).decode().split("\n")[:2]
    sizes = [int(x) for x in a.split()]
    offs = [int(x) for x in b.split()]
    assert sizes == [ctypes.sizeof(A.ImgDesc), ctypes.sizeof(A.AugParams), ctypes.sizeof(A.OutDesc)]
    assert offs == [A.AugParams.lighting.offset, A.AugParams.interp.offset, A.OutDesc.item_stride.offset]


def test_version_and_last_error():
    assert b"gfx950" in A.lib().aeon_hip_version()
    try:
        A.ParamFactory("[")
    except A.AeonHipError as e:
        assert "json" in str(e)


def test_synthetic_generator_is_counter_based():
    a = A.synthetic_image(3, 17, 9)
    b = A.synthetic_image(3, 17, 9)
    c = A.synthetic_image(4, 17, 9)
    assert a.shape == (9, 17, 3) and (a == b).all() and not (a == c).all()
