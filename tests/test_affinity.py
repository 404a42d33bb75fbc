"""CPU: the decode pool's CPU pinning (aeon src/thread_pool.hpp:133-138, src/util.cpp:283-373) for the
product's pool and the CPU baseline's, the per-rank cpu lists bench.py hands each GPU's process,
and the decoder's window draw leaving no trace when a record fails."""
import importlib.util
import os

import pytest

import aeon_amd as A
import oracle as O
from aeon_amd import configs as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALLOWED = sorted(os.sched_getaffinity(0))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _dec(**kw):
    cfg = dict(batch_size=4, random_seed=1, etl=[C.IMAGE_224], augmentation=[C.C2_AUG])
    cfg.update(kw)
    return A.Decoder(cfg)


@pytest.fixture
def no_env_list(monkeypatch):
    monkeypatch.delenv("AEON_CPU_LIST", raising=False)


def test_parse_cpu_list_like_aeon(no_env_list):
    """parse_cpu_list: ranges, sorted, duplicates removed (util.cpp:283-330)."""
    hi = min(ALLOWED[-1], os.cpu_count() - 1)
    assert A.thread_affinity_map("3,0-1,1") == [0, 1, 3] if hi >= 3 else True
    assert A.thread_affinity_map(f"{hi},{hi}") == [hi]


@pytest.mark.parametrize("bad", ["0-100000", "x", "1-y"])
def test_parse_cpu_list_errors(no_env_list, bad):
    with pytest.raises(A.AeonHipError) as e:
        A.thread_affinity_map(bad)
    assert e.value.code == A.AEON_HIP_EINVAL


def test_default_map_is_aeon_policy_over_the_process_mask(no_env_list, monkeypatch):
    """hc - min(2, hc/8) CPUs (util.cpp:360-370), taken from the CPUs this process may run on."""
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    hc = len(ALLOWED)
    assert A.thread_affinity_map() == ALLOWED[:hc - min(2, hc // 8)]


def test_env_list_has_precedence(monkeypatch):
    """AEON_CPU_LIST over the config's cpu_list (util.cpp:344-357)."""
    monkeypatch.setenv("AEON_CPU_LIST", str(ALLOWED[0]))
    assert A.thread_affinity_map(f"{ALLOWED[-1]}") == [ALLOWED[0]]
    d = _dec(cpu_list=f"{ALLOWED[-1]}")
    assert [m for m, _ in d.pool_cpus()] == [ALLOWED[0]]


def test_decoder_workers_report_their_cpus(no_env_list):
    """Every decode-pool worker's own sched_getaffinity holds exactly its map entry."""
    cpus = ALLOWED[::2][:4] if len(ALLOWED) > 1 else ALLOWED
    d = _dec(cpu_list=",".join(map(str, cpus)))
    got = d.pool_cpus()
    assert [m for m, _ in got] == cpus
    assert [w for _, w in got] == [[c] for c in cpus]


def test_decoder_default_pool_is_pinned(no_env_list, monkeypatch):
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    d = _dec()
    got = d.pool_cpus()
    assert [m for m, _ in got] == A.thread_affinity_map()
    assert all(w == [m] for m, w in got)


def test_decode_thread_count_cycles_the_map(no_env_list):
    cpus = ALLOWED[:2]
    d = _dec(cpu_list=",".join(map(str, cpus)), decode_thread_count=5)
    assert [m for m, _ in d.pool_cpus()] == [cpus[i % len(cpus)] for i in range(5)]


def test_oracle_baseline_pool_is_pinned():
    """The CPU baseline's pool pins worker t to map[t % n] like aeon's pool; unpinned after reset."""
    cpus = ALLOWED[:3]
    try:
        O.set_affinity(cpus)
        assert O.pool_cpus(5) == [cpus[t % len(cpus)] for t in range(5)]
    finally:
        O.set_affinity([])
    if len(ALLOWED) > 1:
        assert O.pool_cpus(2) == [-1, -1]


def test_rank_cpu_lists_numa_local_and_disjoint():
    """bench.py --gpus N: each rank's cpu_list lies on its GPU's NUMA node and no two ranks share a
    CPU -- on a two-socket 8-GPU topology, in a container restricted to a few CPUs, and with GPUs
    whose NUMA node is unknown."""
    b = _bench()
    node0, node1 = set(range(0, 64)) | set(range(128, 192)), set(range(64, 128)) | set(range(192, 256))
    local = [node0] * 4 + [node1] * 4
    lists = b.rank_cpu_lists(local, set(range(256)), 8)
    assert len(lists) == 8 and all(lists)
    for r, l in enumerate(lists):
        assert set(l) <= local[r]
        for q in range(r):
            assert not set(l) & set(lists[q])
    assert sum(map(len, lists)) == 256
    # container: 16 CPUs of node 0 only
    allowed = set(range(8)) | set(range(128, 136))
    lists = b.rank_cpu_lists(local, allowed, 8)
    assert all(lists) and all(set(l) <= allowed for l in lists)
    for r in range(8):
        for q in range(r):
            assert not set(lists[r]) & set(lists[q])
    # NUMA node unknown (no sysfs): the allowed CPUs split evenly
    lists = b.rank_cpu_lists([None] * 4, set(range(16)), 4)
    assert lists == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15]]
    # more ranks than CPUs: every rank still gets one (shared), none empty
    lists = b.rank_cpu_lists([None] * 4, {0, 1}, 4)
    assert all(len(l) == 1 for l in lists)


def test_cpu_list_string_round_trip():
    b = _bench()
    assert b.cpu_list_str([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"
    assert A.thread_affinity_map(b.cpu_list_str(ALLOWED[:3])) == ALLOWED[:3] or os.environ.get("AEON_CPU_LIST")


def test_failed_window_draw_leaves_engines(no_env_list):
    """A window whose draw throws (an element of size 0) commits no engine or lighting state: the next
    window's params equal those of a decoder that never saw the failed one."""
    cfg = dict(batch_size=1, random_seed=3, etl=[C.IMAGE_224], augmentation=[C.C3_AUG])
    a, b = A.Decoder(cfg), A.Decoder(cfg)
    sizes = [(300 + i, 260 + i) for i in range(40)]
    bad = list(sizes)
    bad[17] = (0, 260)
    with pytest.raises(A.AeonHipError):
        a.draw_params(bad)
    pa, pb = a.draw_params(sizes), b.draw_params(sizes)
    key = lambda p: (p.crop_x, p.crop_y, p.crop_w, p.crop_h, p.flip, p.hue, p.contrast, tuple(p.lighting[:3]))
    assert [key(p) for p in pa] == [key(p) for p in pb]
