// fuzz_driver.cpp -- runs the host-side parsers of untrusted bytes over a corpus of files, for the
// sanitizer build (aeon_amd/csrc/Makefile target `sanitize`: -fsanitize=address,undefined,
// aeon's SANITIZER_TYPE builds, /root/reference/CMakeLists.txt:80-101).  No device is touched: the
// JPEG entropy decoder (jpeg_host.cpp), the PNG decoder (png_host.cpp) and the JSON reader +
// param_factory (json.hpp, param_factory.cpp) are called directly.
//
// Usage: fuzz_driver FILE...   (*.jpg, *.png, *.json).  One line per file: the outcome, "ok ..." or
// "error <code> <message>"; for a JPEG a second line "gpu<TAB>FILE<TAB>..." with the outcome of the GPU
// entropy decoder's algorithm (jpeg_huff, emulated on the host) on the same bytes.  A sanitizer finding
// aborts the run with a non-zero exit status.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../aeon_amd/csrc/jpeg.hpp"
#include "../../aeon_amd/csrc/param_factory.hpp"
#include "../../include/aeon_hip.h"

namespace aeon_hip {
void jpeg_info(const void* data, size_t size, int* w, int* h, int* ncomp);
void jpeg_entropy_only(const void* data, size_t size, int* w, int* h, int* ncomp, int64_t* n_blocks,
                       int64_t* n_values, uint64_t* hash);
int  jpeg_gpu_entropy_emulate(const void* data, size_t size, int lanes, int* w, int* h, int* ncomp,
                              int64_t* n_blocks, int64_t* n_values, uint64_t* hash, int* rounds);
void png_header(const void* data, size_t size, int* w, int* h, int* depth, int* ctype);
void png_decode(const void* data, size_t size, int mode, void* dst, size_t stride, int* out_elem_bytes);
} // namespace aeon_hip

using namespace aeon_hip;

namespace {

bool ends_with(const std::string& s, const char* suf)
{
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// The GPU entropy decoder's algorithm (host emulation of jpeg_huff) on the same bytes: "gpu host"
// (the file goes to the host decoder), "gpu ok <hash> rounds <r>", "gpu corrupt" or "gpu error <code>".
std::string run_jpeg_gpu(const std::vector<uint8_t>& d)
{
    try {
        int      w, h, n, rounds = 0;
        int64_t  nb, nv;
        uint64_t hv;
        // both workgroup sizes (their subsequence lengths differ: other guessed starts, same result)
        std::string res;
        for (int lanes : {1024, 512, 256}) {
            const int r = jpeg_gpu_entropy_emulate(d.data(), d.size(), lanes, &w, &h, &n, &nb, &nv, &hv, &rounds);
            char      buf[96];
            if (r == 0) std::snprintf(buf, sizeof(buf), "gpu host");
            else if (r < 0) std::snprintf(buf, sizeof(buf), "gpu corrupt");
            else std::snprintf(buf, sizeof(buf), "gpu ok %016llx rounds %d", (unsigned long long)hv, rounds);
            const std::string got = buf, key = got.substr(0, got.find(" rounds"));
            if (res.empty()) res = got;
            else if (res.substr(0, res.find(" rounds")) != key) return "gpu lanes-disagree " + res + " / " + got;
        }
        return res;
    } catch (const jpeg_error& e) {
        return "gpu error " + std::to_string(e.code) + " " + e.what();
    }
}

std::string run_jpeg(const std::vector<uint8_t>& d)
{
    int w, h, n;
    jpeg_info(d.data(), d.size(), &w, &h, &n);
    int64_t  nb, nv;
    uint64_t hv;
    jpeg_entropy_only(d.data(), d.size(), &w, &h, &n, &nb, &nv, &hv);
    char buf[160];
    std::snprintf(buf, sizeof(buf), "ok %dx%dx%d blocks %lld values %lld hash %016llx", w, h, n, (long long)nb,
                  (long long)nv, (unsigned long long)hv);
    return buf;
}

std::string run_png(const std::vector<uint8_t>& d)
{
    int w, h, depth, ctype;
    png_header(d.data(), d.size(), &w, &h, &depth, &ctype);
    if ((int64_t)w * h > (1 << 22)) return "ok header only (large)";
    for (int mode = AEON_PNG_BGR8; mode <= AEON_PNG_ANYDEPTH; mode++) {
        const size_t         stride = (size_t)w * (mode == AEON_PNG_BGR8 ? 3 : 1) * 2;
        std::vector<uint8_t> dst(stride * h);
        int                  eb = 0;
        png_decode(d.data(), d.size(), mode, dst.data(), stride, &eb);
    }
    char buf[96];
    std::snprintf(buf, sizeof(buf), "ok %dx%d depth %d type %d", w, h, depth, ctype);
    return buf;
}

std::string run_json(const std::vector<uint8_t>& d)
{
    const Json    j = Json::parse(std::string(d.begin(), d.end()));
    param_factory f(j);
    std::minstd_rand0 eng(1);
    const int sizes[][2] = {{256, 256}, {1, 1}, {640, 480}, {3, 4000}};
    for (const auto& s : sizes) {
        aeon_aug_params p{};
        f.make_params(eng, s[0], s[1], 224, 224, &p);
    }
    return "ok";
}

} // namespace

int main(int argc, char** argv)
{
    for (int i = 1; i < argc; i++) {
        const std::string    name = argv[i];
        std::ifstream        in(name, std::ios::binary);
        std::vector<uint8_t> d((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        std::string          r, gpu;
        try {
            if (ends_with(name, ".jpg")) {
                gpu = run_jpeg_gpu(d);
                r   = run_jpeg(d);
            }
            else if (ends_with(name, ".png")) r = run_png(d);
            else if (ends_with(name, ".json")) r = run_json(d);
            else r = "skipped";
        } catch (const jpeg_error& e) {
            r = "error " + std::to_string(e.code) + " " + e.what();
        } catch (const std::invalid_argument& e) {
            r = std::string("error -1 ") + e.what();
        } catch (const std::bad_alloc&) {
            r = "error -2 allocation";
        } catch (const std::exception& e) {
            r = std::string("error -2 ") + e.what();
        }
        std::printf("%s\t%s\n", name.c_str(), r.c_str());
        if (!gpu.empty()) std::printf("gpu\t%s\t%s\n", name.c_str(), gpu.c_str());
    }
    return 0;
}
