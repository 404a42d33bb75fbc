"""aeon JSON configurations of the BASELINE.json workloads (SURVEY.md §8(d) config mapping).

C1..C5 are aeon `etl` image/pixelmask objects plus the `augmentation` object, exactly as a
user would hand them to aeon's loader (src/loader.hpp:50-109).
"""
MEAN = [0.485, 0.456, 0.406]
STDDEV = [0.229, 0.224, 0.225]

IMAGE_224 = {"type": "image", "height": 224, "width": 224, "channels": 3, "output_type": "float",
             "channel_major": True, "bgr_to_rgb": True}

C1_AUG = {"type": "image", "center": True, "scale": [0.875, 0.875], "resize_short_size": 256,
          "flip_enable": False, "mean": MEAN, "stddev": STDDEV}
C2_AUG = {"type": "image", "center": False, "scale": [0.5, 1.0], "flip_enable": True,
          "mean": MEAN, "stddev": STDDEV}
C3_AUG = dict(C2_AUG, brightness=[0.5, 1.0], contrast=[0.5, 1.0], saturation=[0.5, 2.0],
              hue=[-18, 18], lighting=[0.0, 0.1])

IMAGE_512 = {"type": "image", "height": 512, "width": 512, "channels": 3, "output_type": "float",
             "channel_major": True, "bgr_to_rgb": True}
MASK_512 = {"type": "pixelmask", "height": 512, "width": 512, "channels": 1, "output_type": "uint8_t"}
C5_AUG = {"type": "image", "center": False, "scale": [0.5, 1.0], "flip_enable": True}

CONFIGS = {
    "C1": {"etl": [IMAGE_224], "augmentation": [C1_AUG], "batch_size": 32},
    "C2": {"etl": [IMAGE_224], "augmentation": [C2_AUG], "batch_size": 256},
    "C3": {"etl": [IMAGE_224], "augmentation": [C3_AUG], "batch_size": 1024},
    "C4": {"etl": [IMAGE_224], "augmentation": [C3_AUG], "batch_size": 1024},
    "C5": {"etl": [IMAGE_512, MASK_512], "augmentation": [C5_AUG], "batch_size": 128},
}


def out_desc_for(etl, aug, item_stride=None):
    """aeon image::config + param_factory mean/stddev -> aeon_amd.OutDesc."""
    import numpy as np

    import aeon_amd as A
    cn = etl.get("channels", 3)
    otype = etl.get("output_type", "uint8_t")
    dtype = {"float": "float32", "uint8_t": "uint8", "int8_t": "int8", "char": "int8", "int16_t": "int16",
             "uint16_t": "uint16", "int32_t": "int32", "uint32_t": "int32", "double": "float64"}[otype]
    esz = np.dtype(A.NP_DTYPE[A.DTYPES[dtype][0]]).itemsize
    mean = aug.get("mean") if etl.get("type") == "image" else None
    std = aug.get("stddev") if etl.get("type") == "image" else None
    if item_stride is None:
        item_stride = etl["height"] * etl["width"] * cn * esz
    return A.out_desc(channels=cn, channel_major=etl.get("channel_major", True),
                      bgr_to_rgb=etl.get("bgr_to_rgb", False), dtype=dtype,
                      mean=mean if mean else None, stddev=std if mean else None,
                      item_stride=item_stride, fixed_aspect_ratio=bool(aug.get("fixed_aspect_ratio", False)),
                      canvas=(etl["width"], etl["height"]))
