"""CPU: the host parsers of untrusted bytes under AddressSanitizer + UndefinedBehaviorSanitizer.

`make -C aeon_amd/csrc sanitize` builds tests/sanitize/fuzz_driver.cpp with the JPEG entropy decoder,
the PNG decoder and the JSON reader + param_factory (aeon's SANITIZER_TYPE builds,
/root/reference/CMakeLists.txt:80-101); it runs over tests/sanitize/corpus.npz (1,749 truncated,
bit-flipped, over-full-table, oversized and deeply nested inputs, tests/sanitize/make_corpus.py).
Every input must end in a clean result or a refused-input error, with no sanitizer report; the
product library (non-sanitized, through the C ABI) must give the same outcome per input.  The driver
also runs the GPU entropy decoder's algorithm (jpeg_huff.hpp's phases, emulated on the host) on every
JPEG: it must produce the host decoder's coefficients bit for bit, or refuse what the host refuses.
"""
import os
import subprocess

import numpy as np
import pytest

import aeon_amd as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "aeon_amd", "csrc", "build_sanitize", "fuzz_driver")


@pytest.fixture(scope="module")
def corpus_run(tmp_path_factory):
    clang = "/opt/rocm/llvm/bin/clang++"
    if not os.path.exists(clang):
        pytest.skip("no clang with sanitizer runtimes")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "aeon_amd", "csrc"), "sanitize"])
    d = tmp_path_factory.mktemp("corpus")
    corpus = np.load(os.path.join(ROOT, "tests", "sanitize", "corpus.npz"))
    names = sorted(corpus.keys())
    for k in names:
        (d / k).write_bytes(corpus[k].tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    env.pop("LD_PRELOAD", None) if "asan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([DRIVER] + [str(d / k) for k in names], capture_output=True, text=True, env=env,
                       timeout=600)
    return r, *_parse(r.stdout), corpus


def _parse(stdout):
    results, gpu = {}, {}
    for line in stdout.splitlines():
        if line.startswith("gpu\t"):
            _, path, res = line.split("\t")
            gpu[os.path.basename(path)] = res
        else:
            path, res = line.split("\t", 1)
            results[os.path.basename(path)] = res
    return results, gpu


def _gpu_agrees(host, gpu):
    """The emulated GPU decoder's outcome against the host decoder's on the same bytes."""
    if gpu == "gpu host":  # progressive / multi-scan: the host decodes it
        return True
    if gpu.startswith("gpu ok"):
        return host.startswith("ok") and host.split("hash ")[1] == gpu.split()[2]
    if gpu == "gpu corrupt":  # corrupt or truncated entropy-coded data
        return host.startswith("error -1 JPEG: corrupt") or host.startswith("error -1 JPEG: truncated scan data")
    return host.startswith("error " + gpu[len("gpu error "):])  # the same header error


def test_corpus_runs_clean_under_asan_ubsan(corpus_run):
    r, results, _, corpus = corpus_run
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert set(results) == set(corpus.keys())
    for k, res in results.items():
        assert res.startswith("ok") or res.startswith("error -1 ") or res.startswith("error -3 "), (k, res)


def test_corpus_expected_outcomes(corpus_run):
    _, results, _, _ = corpus_run
    for k, res in results.items():
        if k.startswith("seed__"):
            assert res.startswith("ok"), (k, res)
        if "__dht_overfull" in k or "__dht_allones" in k:  # jdhuff.c's code-space check
            assert res == "error -1 JPEG: bad Huffman table", (k, res)
        if "__deep_" in k:
            assert res == "error -1 json: nesting too deep", (k, res)
        if k.endswith("__sos_len2_eof.jpg"):
            assert res.startswith("error -1"), (k, res)
    assert sum(r.startswith("ok") for r in results.values()) > 60  # mutations that still decode


def test_product_library_agrees_with_sanitized_driver(corpus_run):
    """The shipped library (aeon_jpeg_entropy_decode / aeon_png_info + aeon_decode_png through the C
    ABI) on the same JPEG / PNG inputs: same accept / refuse decision and error code."""
    _, results, _, corpus = corpus_run
    checked = 0
    for k in sorted(corpus.keys()):
        data = corpus[k].tobytes()
        want = results[k]
        if k.endswith(".jpg"):
            try:
                w, h, n, nb, nv, hv = A.jpeg_entropy_decode(data)
                got = f"ok {w}x{h}x{n} blocks {nb} values {nv} hash {hv:016x}"
            except A.AeonHipError as e:
                got = f"error {e.code}"
            assert got == want if got.startswith("ok") else want.startswith(got + " "), (k, got, want)
            checked += 1
        elif k.endswith(".png"):
            try:
                w, h, depth, ctype = A.png_info(data)
                if w * h <= (1 << 22):
                    for mode in (A.PNG_BGR8, A.PNG_GRAY8, A.PNG_ANYDEPTH):
                        A.decode_png(data, mode)
                got = "ok"
            except A.AeonHipError as e:
                got = f"error {e.code}"
            assert want.startswith(got), (k, got, want)
            checked += 1
    assert checked > 1000


def test_corpus_gpu_entropy_decoder_agrees(corpus_run):
    """jpeg_huff's algorithm (guessed starts, Jacobi rounds, prefix sums, final decode) on every corpus
    JPEG: the host decoder's coefficients bit for bit, or the same refusal."""
    _, results, gpu, corpus = corpus_run
    jpgs = [k for k in corpus.keys() if k.endswith(".jpg")]
    assert set(gpu) == set(jpgs)
    bad = [(k, results[k], gpu[k]) for k in jpgs if not _gpu_agrees(results[k], gpu[k])]
    assert not bad, bad[:5]
    assert sum(g.startswith("gpu ok") for g in gpu.values()) > 100  # decoded on the GPU path
    assert sum(g == "gpu corrupt" for g in gpu.values()) > 10  # corrupt scan data caught


def test_fixtures_gpu_entropy_decoder_bit_exact(tmp_path):
    """aeon's two JPEGs and the synthetic fixtures (4:4:4 / 4:2:2 / 4:2:0 / 4:1:1, restart intervals,
    grayscale, 1x1 .. 600x800, q10 .. q100): every sequential file decodes on the GPU path with the host
    decoder's coefficients; the progressive ones stay on the host."""
    if not os.path.exists("/opt/rocm/llvm/bin/clang++"):
        pytest.skip("no clang with sanitizer runtimes")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "aeon_amd", "csrc"), "sanitize"])
    fx = np.load(os.path.join(ROOT, "tests", "golden", "jpeg_fixtures.npz"))
    names = [k for k in fx.files if k.endswith(".jpg")]
    for k in names:
        (tmp_path / k).write_bytes(fx[k].tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:exitcode=86")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([DRIVER] + [str(tmp_path / k) for k in names], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    results, gpu = _parse(r.stdout)
    for k in names:
        if k.startswith("prog_"):
            assert gpu[k] == "gpu host", (k, gpu[k])
        else:
            assert gpu[k].startswith("gpu ok") and _gpu_agrees(results[k], gpu[k]), (k, results[k], gpu[k])


HOST_ASAN = os.path.join(ROOT, "aeon_amd", "csrc", "build_sanitize", "host_driver_asan")
HOST_TSAN = os.path.join(ROOT, "aeon_amd", "csrc", "build_sanitize", "host_driver_tsan")


def _host_driver(target, exe, env_extra):
    """tests/sanitize/host_driver.cpp over host.cpp + stager.cpp with the HIP runtime stubbed
    (tests/sanitize/hip_stubs.cpp): loader configs, the pinned thread_pool, window draws on the pool
    against serial draws over odd and even windows, a failing window, concurrent stager stages."""
    if not os.path.exists("/opt/rocm/llvm/bin/clang++"):
        pytest.skip("no clang with sanitizer runtimes")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "aeon_amd", "csrc"), target])
    env = dict(os.environ, **env_extra)
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, "2"], capture_output=True, text=True, env=env, timeout=900)
    lines = [l for l in r.stdout.splitlines() if "\t" in l]
    return r, lines


def test_host_layer_under_asan_ubsan():
    r, lines = _host_driver("sanitize", HOST_ASAN, {"ASAN_OPTIONS": "detect_leaks=1:exitcode=86",
                                                    "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1:exitcode=87"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert len(lines) >= 20 and all("\tok" in l for l in lines), r.stdout


def test_host_layer_under_tsan():
    """aeon's SANITIZER_TYPE=Thread build (/root/reference/CMakeLists.txt:80-101) of the pool code:
    the draws of a window on the pool, pools started and stopped back to back, concurrent stages."""
    r, lines = _host_driver("tsan", HOST_TSAN, {"TSAN_OPTIONS": "halt_on_error=1:exitcode=66"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert len(lines) >= 20 and all("\tok" in l for l in lines), r.stdout
