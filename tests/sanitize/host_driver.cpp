// host_driver.cpp -- the decoder's host layer (aeon_amd/csrc/host.cpp) under AddressSanitizer +
// UndefinedBehaviorSanitizer and under ThreadSanitizer (aeon's SANITIZER_TYPE builds,
// /root/reference/CMakeLists.txt:80-101), linked against tests/sanitize/hip_stubs.cpp instead of the
// HIP runtime.  What runs: loader-config parsing and verify_config (valid and malformed configs),
// provider_factory, the pinned thread_pool (creation, pinning, teardown, first-exception rethrow), the
// window draws on the pool (draw_window: every record on the pool with its slot engine, the lighting
// cache fixed up in order) against the serial draws over odd and even windows, a window that throws
// (an element of size 0) and the windows after it, the node slicing, and cpu lists.
//
// Usage: host_driver [rounds]   One line per case, "name<TAB>ok ..." or "name<TAB>FAIL ..."; exit 1 if
// any case failed (a sanitizer finding aborts the run with its own exit status).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/aeon_hip.h"

namespace {

int failures = 0;

void report(const std::string& name, bool ok, const std::string& what)
{
    std::printf("%s\t%s %s\n", name.c_str(), ok ? "ok" : "FAIL", what.c_str());
    if (!ok) failures++;
}

const char* kImage224 =
    R"({"type": "image", "height": 224, "width": 224, "channels": 3, "output_type": "float", "channel_major": true, "bgr_to_rgb": true})";
const char* kC2Aug =
    R"({"type": "image", "scale": [0.5, 1.0], "flip_enable": true, "mean": [0.485, 0.456, 0.406], "stddev": [0.229, 0.224, 0.225]})";
const char* kC3Aug =
    R"({"type": "image", "scale": [0.5, 1.0], "flip_enable": true, "mean": [0.485, 0.456, 0.406], "stddev": [0.229, 0.224, 0.225], "brightness": [0.5, 1.0], "contrast": [0.5, 1.0], "saturation": [0.5, 2.0], "hue": [-18, 18], "lighting": [0.0, 0.1]})";
const char* kMask512 = R"({"type": "pixelmask", "height": 512, "width": 512, "channels": 1, "output_type": "uint8_t"})";
const char* kImage512 =
    R"({"type": "image", "height": 512, "width": 512, "channels": 3, "output_type": "float", "channel_major": true, "bgr_to_rgb": true})";

std::string loader(const std::string& etl, const std::string& aug, const std::string& extra)
{
    return R"({"batch_size": 4, "random_seed": 7, "etl": [)" + etl + R"(], "augmentation": [)" + aug + "]" + extra + "}";
}

struct Records {
    std::vector<uint8_t>          pixel{0};
    std::vector<aeon_record_elem> elems;
    Records(int n, int ne, unsigned seed, int bad = -1)
    {
        for (int i = 0; i < n; i++) {
            seed      = seed * 1103515245u + 12345u;
            const int w = 120 + (int)(seed >> 16) % 500, h = 100 + (int)(seed >> 8) % 500;
            for (int k = 0; k < ne; k++)
                elems.push_back(aeon_record_elem{pixel.data(), i == bad ? 0 : w, h, k == 0 ? 3 : 1, 0});
        }
    }
};

bool same_params(const std::vector<aeon_aug_params>& a, const std::vector<aeon_aug_params>& b)
{
    return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(aeon_aug_params)) == 0;
}

// draw windows on the pool (decoder a) and serially (decoder b) from the same slot engines
void draw_windows(const std::string& name, const std::string& cfg, int ne, int rounds)
{
    aeon_decoder *a = nullptr, *b = nullptr;
    if (aeon_decoder_create(cfg.c_str(), 0, &a) || aeon_decoder_create(cfg.c_str(), 0, &b)) {
        report(name, false, std::string("create: ") + aeon_decoder_last_error());
        return;
    }
    int  workers = 0;
    bool ok      = aeon_decoder_pool_size(a, &workers) == 0 && workers > 0;
    for (int w = 0; ok && w < workers; w++) {
        int map_cpu = -2, cpus[1024], count = 0;
        ok = aeon_decoder_pool_cpus(a, w, &map_cpu, cpus, 1024, &count) == 0 && count > 0;
    }
    const int windows[] = {5, 130, 33, 64, 1, 257};
    unsigned  seed      = 11;
    for (int r = 0; ok && r < rounds; r++)
        for (int n : windows) {
            Records                      recs(n, ne, seed++);
            std::vector<aeon_aug_params> pa(n), pb(n);
            ok = ok && aeon_decoder_draw_params(a, n, recs.elems.data(), pa.data(), 0) == 0 &&
                 aeon_decoder_draw_params(b, n, recs.elems.data(), pb.data(), 1) == 0 && same_params(pa, pb);
        }
    report(name, ok, "pool " + std::to_string(workers) + " workers, parallel draws == serial draws");
    aeon_decoder_destroy(a);
    aeon_decoder_destroy(b);
}

// a window whose draw throws on the pool leaves the decoder's engines and lighting cache untouched
void failed_window(const std::string& name, const std::string& cfg)
{
    aeon_decoder *a = nullptr, *b = nullptr;
    aeon_decoder_create(cfg.c_str(), 0, &a);
    aeon_decoder_create(cfg.c_str(), 0, &b);
    Records                      bad(40, 1, 3, 17), good(40, 1, 4);
    std::vector<aeon_aug_params> pa(40), pb(40);
    const int                    rc = aeon_decoder_draw_params(a, 40, bad.elems.data(), pa.data(), 0);
    const std::string            msg = aeon_decoder_last_error();
    bool ok = rc == AEON_HIP_ERUNTIME && msg.find("with size 0") != std::string::npos;
    ok      = ok && aeon_decoder_draw_params(a, 40, good.elems.data(), pa.data(), 0) == 0 &&
         aeon_decoder_draw_params(b, 40, good.elems.data(), pb.data(), 0) == 0 && same_params(pa, pb);
    report(name, ok, "rc " + std::to_string(rc) + " (" + msg + ")");
    aeon_decoder_destroy(a);
    aeon_decoder_destroy(b);
}

void invalid_config(const std::string& name, const std::string& cfg, int want)
{
    aeon_decoder* d  = nullptr;
    const int     rc = aeon_decoder_create(cfg.c_str(), 0, &d);
    report(name, rc == want && !d, "rc " + std::to_string(rc) + " (" + aeon_decoder_last_error() + ")");
    if (d) aeon_decoder_destroy(d);
}

} // namespace

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 2;
    const std::string c2 = loader(kImage224, kC2Aug, ""), c3 = loader(kImage224, kC3Aug, "");
    draw_windows("draw_c2", c2, 1, rounds);
    draw_windows("draw_c3_lighting", c3, 1, rounds);
    draw_windows("draw_c5_image_mask", loader(std::string(kImage512) + ", " + kMask512, kC2Aug, ""), 2, rounds);
    draw_windows("draw_c3_cpu_list", loader(kImage224, kC3Aug, R"(, "cpu_list": "0")"), 1, rounds);
    draw_windows("draw_c3_thread_count", loader(kImage224, kC3Aug, R"(, "decode_thread_count": 5)"), 1, rounds);
    draw_windows("draw_c3_node", loader(kImage224, kC3Aug, R"(, "node_id": 3, "node_count": 8)"), 1, rounds);
    failed_window("failed_window_c3", c3);
    failed_window("failed_window_c2", c2);

    // pools started and stopped back to back (thread start-up, pinning and shutdown races)
    bool ok = true;
    for (int i = 0; i < 20 * rounds; i++) {
        aeon_decoder* d = nullptr;
        ok = ok && aeon_decoder_create(c3.c_str(), 0, &d) == 0;
        int w = 0;
        if (d && i % 2) ok = ok && aeon_decoder_pool_size(d, &w) == 0;
        aeon_decoder_destroy(d);
    }
    report("pool_lifecycle", ok, std::to_string(20 * rounds) + " decoders");

    // a decode window needs the device: the stub refuses it and the decoder stays usable
    {
        aeon_decoder* d = nullptr;
        aeon_decoder_create(c2.c_str(), 0, &d);
        Records recs(4, 1, 9);
        std::vector<float> out(4 * 3 * 224 * 224);
        void*              outs[1] = {out.data()};
        const int          rc = aeon_decoder_decode(d, 4, recs.elems.data(), outs, 0, nullptr);
        std::vector<aeon_aug_params> p(4);
        const std::string msg = aeon_decoder_last_error();
        report("decode_without_device",
               rc == AEON_HIP_ERUNTIME && msg.find("no device") != std::string::npos &&
                   aeon_decoder_draw_params(d, 4, recs.elems.data(), p.data(), 0) == 0,
               "rc " + std::to_string(rc) + " (" + msg + ")");
        aeon_decoder_destroy(d);
    }

    // the aeon-side stager: 8 threads stage 4 batches concurrently (pinned chunk bump allocation,
    // per-batch slots); the window's flush fails without a device and drops the window whole; the
    // next window's stages work
    {
        aeon_out_desc o{};
        o.dtype = AEON_DTYPE_F32, o.channels = 3, o.channel_major = 1, o.item_stride = 3 * 224 * 224 * 4;
        aeon_hip_stager* st  = nullptr;
        const int        rc0 = aeon_hip_stager_create(reinterpret_cast<aeon_hip_ctx*>(0x10), AEON_STAGER_IMAGE, &o, 16, &st);
        std::vector<uint8_t>  px(300 * 200 * 3, 7);
        std::vector<std::vector<float>> outs(4, std::vector<float>(16 * 3 * 224 * 224));
        aeon_aug_params p{};
        p.crop_w = 200, p.crop_h = 150, p.out_w = 224, p.out_h = 224, p.contrast = p.brightness = p.saturation = 1.f;
        bool ok = rc0 == 0;
        for (int window = 0; ok && window < 2; window++) {
            std::vector<std::thread> th;
            std::vector<int>         rcs(64, -99);
            for (int t = 0; t < 8; t++)
                th.emplace_back([&, t] {
                    for (int i = t; i < 64; i += 8)
                        rcs[i] = aeon_hip_stager_stage(st, outs[i / 16].data(), i % 16, px.data(), 300, 200, 0, 3, 1, &p);
                });
            for (auto& x : th) x.join();
            for (int r : rcs)
                if (r != 0) ok = false, std::printf("stage rc %d: %s\n", r, aeon_hip_stager_last_error());
            const int rf = aeon_hip_stager_flush(st, outs[0].data()); // no device: the launch fails
            if (rf == 0) ok = false, std::printf("flush without a device succeeded\n");
        }
        report("stager_concurrent_stage", ok, "rc " + std::to_string(rc0) + " (" + aeon_hip_stager_last_error() + ")");
        aeon_hip_stager_destroy(st);
    }

    invalid_config("config_not_json", "{\"batch_size\": 4, ", AEON_HIP_EINVAL);
    invalid_config("config_unknown_key", loader(kImage224, kC2Aug, R"(, "shuffle_manifst": true)"), AEON_HIP_EINVAL);
    invalid_config("config_no_batch", R"({"etl": [{"type": "image", "height": 8, "width": 8}]})", AEON_HIP_EINVAL);
    invalid_config("config_bad_etl", loader(R"({"type": "image", "height": 8, "width": 8, "channels": 2})", kC2Aug, ""),
                   AEON_HIP_EINVAL);
    invalid_config("config_bad_cpu_list", loader(kImage224, kC2Aug, R"(, "cpu_list": "0-100000")"), AEON_HIP_EINVAL);
    invalid_config("config_cpu_list_text", loader(kImage224, kC2Aug, R"(, "cpu_list": "a-b")"), AEON_HIP_EINVAL);
    invalid_config("config_zero_threads", loader(kImage224, kC2Aug, R"(, "decode_thread_count": 0)"), AEON_HIP_EINVAL);
    invalid_config("config_node", loader(kImage224, kC2Aug, R"(, "node_id": 8, "node_count": 8)"), AEON_HIP_ERUNTIME);
    invalid_config("config_deep", std::string(300, '[') + std::string(300, ']'), AEON_HIP_EINVAL);

    {
        int cpus[64], n = 0;
        const bool a = aeon_thread_affinity_map("2,0-1,1", cpus, 64, &n) == 0 && n == 3 && cpus[0] == 0 && cpus[2] == 2;
        const bool b = aeon_thread_affinity_map("0-99999", cpus, 64, &n) == AEON_HIP_EINVAL;
        const bool c = aeon_thread_affinity_map("", cpus, 0, &n) == 0 && n > 0;
        report("cpu_lists", a && b && c, "");
    }
    {
        int64_t idx[4096], cnt = 0;
        bool    ok2 = aeon_manifest_node_slice(4096, 256, 3, 8, idx, &cnt) == 0 && cnt == 512 && idx[0] == 768;
        ok2 = ok2 && aeon_manifest_node_slice(257, 7, 2, 3, nullptr, &cnt) == 0 && cnt == 85;
        ok2 = ok2 && aeon_manifest_node_slice(10, 2, 5, 2, idx, &cnt) == AEON_HIP_EINVAL;
        report("node_slices", ok2, "");
    }
    return failures ? 1 : 0;
}
