"""Generate the committed golden fixtures from aeon's own test data.

Run in the dev container only (it reads /root/reference, which does not exist on
the GPU box); the outputs are committed so tests never touch the reference.

Fixtures written (all data, no reference source):
  img_2112_70_bgr.npz        decoded test/test_data/img_2112_70.jpg as HWC BGR uint8
                             (480x360x3).  Decoded with Pillow (libjpeg-turbo, ISLOW
                             IDCT, fancy upsampling) -- the same decoder settings
                             OpenCV's imdecode uses; validated by the goldens below.
  augment_output_linear.npz  the two fp32 CHW RGB goldens used by
                             test/test_provider.cpp:96-261
                             (provider.image_paddle_imagenet_{training,validate}_augmentation)
                             stored verbatim as float32 [3,224,224].
"""
import hashlib
import os
import sys

import numpy as np

REF = "/root/reference/test/test_data"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    from PIL import Image  # dev-container only

    jpg = os.path.join(REF, "img_2112_70.jpg")
    rgb = np.asarray(Image.open(jpg).convert("RGB"), dtype=np.uint8)
    bgr = np.ascontiguousarray(rgb[:, :, ::-1])
    assert bgr.shape == (360, 480, 3), bgr.shape
    np.savez_compressed(os.path.join(HERE, "img_2112_70_bgr.npz"), bgr=bgr,
                        sha256=np.frombuffer(hashlib.sha256(bgr.tobytes()).digest(), np.uint8))

    out = {}
    for name in ("train", "eval"):
        raw = np.fromfile(os.path.join(REF, f"augment_output_linear_{name}.bin"), dtype=np.float32)
        assert raw.size == 3 * 224 * 224, raw.size
        out[name] = raw.reshape(3, 224, 224)
    np.savez_compressed(os.path.join(HERE, "augment_output_linear.npz"), **out)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
