// Host cost of param_factory::make_params per decode window (the decoder draws in record order on
// its own thread, host.cpp batch_decoder::enqueue): aeon_make_params for 1024 records of each
// configuration's augmentation, median of 20 windows.  Host only (no GPU).
//   g++ -O2 -std=c++17 -I include tools/make_params_timing.cpp -L aeon_amd -laeon_hip -Wl,-rpath,$PWD/aeon_amd
#include <aeon_hip.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

int main()
{
    const char* cfgs[][2] = {
        {"C1", R"({"type":"image","center":true,"scale":[0.875,0.875],"resize_short_size":256,"flip_enable":false})"},
        {"C2", R"({"type":"image","center":false,"scale":[0.5,1.0],"flip_enable":true})"},
        {"C3", R"({"type":"image","center":false,"scale":[0.5,1.0],"flip_enable":true,"brightness":[0.5,1.0],)"
               R"("contrast":[0.5,1.0],"saturation":[0.5,2.0],"hue":[-18,18],"lighting":[0.0,0.1]})"},
    };
    const int n = 1024;
    for (auto& c : cfgs) {
        aeon_param_factory* f = nullptr;
        if (aeon_param_factory_create(c[1], &f) != 0) {
            std::printf("%s: create failed\n", c[0]);
            return 1;
        }
        std::vector<uint32_t>        st(n);
        std::vector<aeon_aug_params> out(n);
        for (int i = 0; i < n; i++) st[i] = 12345u + i;
        std::vector<double> us;
        for (int w = 0; w < 20; w++) {
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; i++) aeon_make_params(f, &st[i], 256, 256, 224, 224, &out[i]);
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(us.begin(), us.end());
        std::printf("%s: make_params x %d records: median %.1f us per window (%.3f us per record)\n", c[0], n, us[10],
                    us[10] / n);
        aeon_param_factory_destroy(f);
        // the decoder's draw phase of a 1024-record window: in record order vs on its pool
        const std::string dcfg = std::string(R"({"batch_size":32,"random_seed":1,"etl":[{"type":"image","height":224,)"
                                             R"("width":224,"channels":3}],"augmentation":[)") + c[1] + "]}";
        aeon_decoder* d = nullptr;
        if (aeon_decoder_create(dcfg.c_str(), 0, &d) != 0) {
            std::printf("%s: decoder create failed: %s\n", c[0], aeon_decoder_last_error());
            return 1;
        }
        static uint8_t                px = 0;
        std::vector<aeon_record_elem> el(n, aeon_record_elem{&px, 256, 256, 3, 768});
        for (int serial = 1; serial >= 0; serial--) {
            std::vector<double> ds;
            for (int w = 0; w < 21; w++) {
                auto t0 = std::chrono::steady_clock::now();
                aeon_decoder_draw_params(d, n, el.data(), out.data(), serial);
                ds.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            }
            std::sort(ds.begin(), ds.end());
            std::printf("%s: decoder window draw x %d records, %s: median %.1f us\n", c[0], n,
                        serial ? "in record order" : "on the pool", ds[10]);
        }
        aeon_decoder_destroy(d);
    }
    return 0;
}
