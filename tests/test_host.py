"""CPU: the host provider surface (provider_factory / image::config / loader keys) and aeon's
manifest node slicing, including a 2-rank gloo run of the per-GPU slicing."""
import os

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C


def _dec(**kw):
    cfg = dict(batch_size=4, random_seed=1, etl=[C.IMAGE_224], augmentation=[C.C2_AUG])
    cfg.update(kw)
    return A.Decoder(cfg)


def test_output_shapes():
    d = A.Decoder(dict(batch_size=8, etl=[dict(C.IMAGE_512, name="left"), C.MASK_512],
                       augmentation=[C.C5_AUG]))
    assert [o["name"] for o in d.outputs] == ["left.image", "pixelmask"]
    assert d.outputs[0]["shape"] == (3, 512, 512) and d.outputs[0]["dtype"] == np.float32
    assert d.outputs[1]["shape"] == (1, 512, 512) and d.outputs[1]["item_bytes"] == 512 * 512
    hwc = A.Decoder(dict(batch_size=1, etl=[dict(C.IMAGE_224, channel_major=False, output_type="uint8_t")]))
    assert hwc.outputs[0]["shape"] == (224, 224, 3)


@pytest.mark.parametrize("bad", [
    dict(etl=[dict(C.IMAGE_224, heigth=224)]),                 # unknown image key (verify_config)
    dict(etl=[dict(C.IMAGE_224, channels=2)]),                 # channels must be 1 or 3
    dict(etl=[dict(C.IMAGE_224, channels=1)]),                 # bgr_to_rgb needs 3 channels
    dict(etl=[dict(C.IMAGE_224, output_type="float16")]),      # not an aeon output type
    dict(etl=[dict(C.IMAGE_224, output_type="uint8_t")]),      # mean/stddev need float output
    dict(etl=[{"height": 10, "width": 10}]),                   # etl object without type
    dict(etl=[dict(C.IMAGE_224, type="videoo")]),              # unsupported etl type
    dict(shuffle_manifst=True),                                # unknown loader key
    dict(augmentation=[{"scale": [0.5, 1.0]}]),                # augmentation without type
    dict(augmentation=[dict(C.C2_AUG, mean=[0.5, 0.5])]),      # mean size != channels
    dict(etl=[dict(C.IMAGE_224, width=0)]),
])
def test_invalid_configs(bad):
    with pytest.raises(A.AeonHipError) as e:
        _dec(**bad)
    assert e.value.code in (A.AEON_HIP_EINVAL, A.AEON_HIP_ERUNTIME)


def test_missing_batch_size():
    with pytest.raises(A.AeonHipError):
        A.Decoder(dict(etl=[C.IMAGE_224]))


def test_node_id_out_of_range():
    with pytest.raises(A.AeonHipError):
        _dec(node_id=2, node_count=2)


def _ref_slice(n, b, node, nodes):
    """aeon manifest_file::generate_blocks node slicing, restated (manifest_file.cpp:278-295)."""
    if nodes <= 1:
        return list(range(n))
    cnt = n // nodes
    batches = cnt // b
    out = [(i // b) * b * nodes + b * node + i % b for i in range(batches * b)]
    tail = cnt - batches * b
    out += [batches * b * nodes + tail * node + i for i in range(tail)]
    return out


@pytest.mark.parametrize("n,b,nodes", [(10, 2, 2), (1000, 32, 8), (257, 7, 3), (5, 8, 2), (4096, 256, 8)])
def test_manifest_node_slice(n, b, nodes):
    seen = []
    for node in range(nodes):
        s = A.manifest_node_slice(n, b, node, nodes)
        assert list(s) == _ref_slice(n, b, node, nodes)
        seen += list(s)
    assert len(seen) == len(set(seen))  # disjoint slices
    assert all(0 <= i < n for i in seen)


def test_manifest_interleave_like_aeon_test():
    """test/test_manifest_tsv.cpp:113-205: two nodes take alternate batches."""
    a = A.manifest_node_slice(8, 2, 0, 2)
    b = A.manifest_node_slice(8, 2, 1, 2)
    assert list(a) == [0, 1, 4, 5] and list(b) == [2, 3, 6, 7]


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = torch.from_numpy(A.manifest_node_slice(4096, 256, rank, world))
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    if rank == 0:
        q.put(sorted(torch.cat(allv).tolist()))
    dist.destroy_process_group()


def test_gloo_two_ranks_cover_the_manifest():
    """The bench's N-GPU sharding, rehearsed on CPU: each rank owns one aeon node slice; the
    slices of all ranks are disjoint and cover every full batch of the manifest."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == list(range(4096))


def test_bench_launcher_dry_run_two_ranks():
    """`bench.py --gpus 2` starts torchrun itself (a child process) and every rank takes its aeon
    node slice (manifest_file.cpp:278-295) and decoder seed random_seed + node_id (loader.cpp:174):
    rehearsed with gloo and a stub workload, checked against the restated slicing and seeding."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and len(line["ranks"]) == 2
    b, n = line["batch_per_rank"], line["n_records"]
    for info in line["ranks"]:
        rk = info["rank"]
        assert info["node_id"] == rk and info["seed"] == 1 + rk
        ref = _ref_slice(n, b, rk, 2)
        assert info["slice_len"] == len(ref) and info["slice_head"] == ref[:2 * b]
        assert info["slot_states"] == list(A.seed_slots(1 + rk, 4))
    assert line["ranks"][0]["slot_states"] != line["ranks"][1]["slot_states"]
    # each rank's decode-pool cpu_list (AEON_CPU_LIST): non-empty, allowed, disjoint across ranks
    lists = [set(A.thread_affinity_map(info["cpu_list"])) for info in line["ranks"]]
    assert all(lists) and all(l <= set(os.sched_getaffinity(0)) for l in lists)
    if len(os.sched_getaffinity(0)) >= 2:
        assert not lists[0] & lists[1]


def test_bench_synthetic_pool_matches_synthetic_image():
    """The bench's device pixel generator is A.synthetic_image (splitmix64 per record index)."""
    import torch
    sys_path_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(sys_path_root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    recs = [0, 7, 4097, 123456]
    pool = bench.synthetic_pool(torch, recs, 19, 11, device="cpu", chunk=3).numpy()
    L = 19 * 11 * 3
    for k, g in enumerate(recs):
        assert np.array_equal(pool[k * L:(k + 1) * L], A.synthetic_image(g, 19, 11, 3).reshape(-1))


def _param_tuple(p):
    return (p.crop_x, p.crop_y, p.crop_w, p.crop_h, p.flip, p.angle, p.hue, p.contrast, p.brightness,
            p.saturation, tuple(p.lighting[:3]), p.n_lighting)


@pytest.mark.parametrize("aug_name", ["C2", "C3"])
def test_decoder_draw_window_matches_in_order_draws(aug_name):
    """batch_decoder's parallel window draw (draw_window: every record on the pool with its slot
    engine, the lighting normal_distribution's cached value handed on in one in-order pass) gives
    the params of aeon's in-order draws: the decoder's own serial loop, and the oracle's factory
    whose libstdc++ normal_distribution keeps the cache itself.  Windows of odd and even sizes so
    the cache is both empty and full at window starts (batch_decoder.cpp:62-71)."""
    from tests import helpers as H
    import oracle as O
    aug = {"C2": C.C2_AUG, "C3": C.C3_AUG}[aug_name]
    cfg = dict(batch_size=1, random_seed=7, etl=[C.IMAGE_224], augmentation=[aug])
    par, ser = A.Decoder(cfg), A.Decoder(cfg)
    fac = O.Factory(H.oracle_aug_config(aug))
    windows = [5, 130, 33, 64, 1]
    states = O.seed_slots(7, max(windows))
    rng = np.random.default_rng(3)
    for n in windows:
        sizes = [(int(rng.integers(200, 600)), int(rng.integers(200, 600))) for _ in range(n)]
        a = par.draw_params(sizes, serial=False)
        b = ser.draw_params(sizes, serial=True)
        ref = []
        for i, (w, h) in enumerate(sizes):
            st = states[i:i + 1]
            ref.append(fac.make_params(st, w, h, 224, 224))
            states[i] = st[0]
        for i in range(n):
            assert _param_tuple(a[i]) == _param_tuple(b[i]), (n, i)
            r = ref[i]
            assert (a[i].crop_x, a[i].crop_y, a[i].crop_w, a[i].crop_h, a[i].flip, a[i].hue) == \
                (r.crop_x, r.crop_y, r.crop_w, r.crop_h, r.flip, r.hue), (n, i)
            assert (a[i].contrast, a[i].brightness, a[i].saturation) == (r.contrast, r.brightness, r.saturation)
            assert tuple(a[i].lighting[:3]) == tuple(r.lighting[:3]), (n, i)
    if aug_name == "C3":
        assert any(p.lighting[0] != 0 for p in a)
