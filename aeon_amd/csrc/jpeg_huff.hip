// jpeg_huff.hip -- GPU Huffman decoding of sequential JPEG scans (ITU T.81 F.2.2; libjpeg's jdhuff.c
// decode_mcu as cv::imdecode runs it under aeon's image::extractor::extract, src/etl_image.cpp:83-99),
// for the files jpeg_host.cpp hands over whole: one scan carrying every component, its entropy-coded
// bytes unstuffed and split at RSTn markers into segments (restart intervals) by the host.
//
// One workgroup per file.  A segment's bits are cut into subsequences of F.sub_bits; the decoder
// state at a codeword boundary is (bit position, block within the MCU c, zigzag index k), and the
// state at a subsequence's end is a function of the state at its start.  So:
//   1. every subsequence is decoded from a guessed start (its first bit, c = 0, k = 0; the segment's
//      first subsequence starts exactly) up to the first codeword boundary at or past its end;
//   2. Jacobi rounds: a subsequence whose start differs from its predecessor's end takes that end as
//      its start and is decoded again -- until no start changes.  The segment's first start is exact,
//      so after round r the first r + 1 starts are; Huffman codes (and JPEG's block structure)
//      re-synchronise within a few codewords, so two or three rounds settle a file in practice;
//   3. with exact starts, an exclusive prefix sum over the subsequences gives each one its first
//      block and its DC predictors (blocks started, DC differences per component);
//   4. a final decode of each subsequence writes its coefficients into the dense block slots (64 int16
//      per block, zigzag order) and the blocks' non-zero masks, which jpeg_idct reads.
// Decoding tables live in LDS: a kHuffFastBits lookahead per table whose entries carry the code
// length, the AC run and, when the value bits fit the lookahead too, the decoded value; longer codes
// take the canonical maxcode walk.  The bit reader holds 64 bits and one word loaded ahead, so the
// next refill's global load is in flight while the current bits decode.  A file with at most one
// subsequence per lane keeps each lane's subsequence state in registers (decode_lanes).  The per-lane logic is in
// jpeg_huff.hpp (shared with the host emulation the CPU tests run).
#include <hip/hip_runtime.h>

#include "jpeg_huff.hpp"

namespace aeon_hip {
namespace {

// AEON_HUFF_PROBE builds (tools/build_variants.sh, development only): lane 0 of workgroup 0 stamps
// the wall clock (100 MHz) at the phase boundaries of its file and prints them at the end.
#ifdef AEON_HUFF_PROBE
__shared__ unsigned long long probe_t[256];
__shared__ int                probe_n[256];
__shared__ int                probe_k;
#define HUFF_STAMP(what, n)                                                                                   \
    do {                                                                                                      \
        if (blockIdx.x == 0 && threadIdx.x == 0 && probe_k < 256)                                             \
            probe_t[probe_k] = wall_clock64(), probe_n[probe_k++] = (int)(n);                                 \
    } while (0)
#else
#define HUFF_STAMP(what, n) \
    do {                    \
        (void)(n);          \
    } while (0)
#endif

struct Scan {
    int4 wsum[1024 / 64];
    int4 carry;
};

// Inclusive scan of v over the workgroup's LANES lanes, plus the running carry of earlier chunks.
template <int LANES>
__device__ int4 wg_scan(Scan& X, int4 v)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(v.x, o), y = __shfl_up(v.y, o), z = __shfl_up(v.z, o), w = __shfl_up(v.w, o);
        if (lane >= o) v.x += x, v.y += y, v.z += z, v.w += w;
    }
    if (lane == 63) X.wsum[wave] = v;
    __syncthreads();
    int4 off = X.carry;
    for (int i = 0; i < wave; i++) off.x += X.wsum[i].x, off.y += X.wsum[i].y, off.z += X.wsum[i].z, off.w += X.wsum[i].w;
    v.x += off.x, v.y += off.y, v.z += off.z, v.w += off.w;
    __syncthreads();
    if (threadIdx.x == LANES - 1) X.carry = v;
    return v;
}

} // namespace

typedef __attribute__((address_space(1))) JpegHuffSub glb_sub;

// A file with more subsequences than lanes: the phases over the subsequence states in F.subs.
template <int LANES>
__device__ __forceinline__ void decode_strided(const huff::Tables& T, Scan& X, const JpegHuffFile& F, int32_t* error)
{
    const int tid = threadIdx.x, nsub = F.nsub;
    glb_sub*  subs = (glb_sub*)F.subs;
    // 1. guessed starts; 2. Jacobi rounds until every start is its predecessor's end
    huff::pass_guess(T, F, subs, tid, LANES);
    for (;;) {
        __syncthreads();
        const int any = huff::pass_compare(F, subs, tid, LANES);
        if (!__syncthreads_or(any)) break;
        huff::pass_rewalk(T, F, subs, tid, LANES);
    }
    // 3. exclusive prefix of (blocks, DC differences) over the file's subsequences
    for (int base = 0; base < nsub; base += LANES) {
        const int  j = base + tid;
        const int4 v = j < nsub ? make_int4(subs[j].cnt[0], subs[j].cnt[1], subs[j].cnt[2], subs[j].cnt[3])
                                : make_int4(0, 0, 0, 0);
        const int4 s = wg_scan<LANES>(X, v);
        if (j < nsub) subs[j].ex[0] = s.x - v.x, subs[j].ex[1] = s.y - v.y, subs[j].ex[2] = s.z - v.z, subs[j].ex[3] = s.w - v.w;
        __syncthreads();
    }
    // 4. the final decode: coefficients and masks
    if (!huff::pass_write(T, F, subs, tid, LANES)) atomicOr(error, kJpegCorruptBit);
}

// LDS of a file with at most LANES subsequences: each one's end state, walk bounds (stop, segment end)
// and counts (exclusive sums after the prefix), and a round's list of subsequences to walk again.
template <int LANES>
struct LaneStates {
    uint64_t en[LANES];
    uint2    se[LANES];
    int4     ex[LANES];
    int      todo[LANES];
    int      wave_n[LANES / 64];
};

// A file with at most one subsequence per lane (the common case): lane j owns subsequence j (its
// segment and start state in registers) for the guessed start and the final decode.  A Jacobi round
// compacts the subsequences whose start changed into the first lanes (wave ballots), so the walks of
// a round occupy ceil(changed / 64) waves instead of every wave holding one.  The same phases as
// jpeg_huff.hpp's pass_* functions, which the host emulation checks.
template <int LANES, typename WP>
__device__ __forceinline__ void decode_lanes(const huff::Tables& T, Scan& X, LaneStates<LANES>& L,
                                             const JpegHuffFile& F, WP words, int32_t* error)
{
    const int  tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nsub = F.nsub;
    const bool have = tid < nsub;
    int        sg = 0, i = 0;
    JpegHuffSeg S{0, 0, 0, 1};
    if (have) {
        sg = huff::gmem<const int32_t>(F.sub_seg)[tid];
        S  = huff::gmem<const JpegHuffSeg>(F.segs)[sg];
        i  = tid - S.first_sub;
    }
    const bool first = i == 0, last = i + 1 == S.nsub;
    const int  p0    = (int)S.start_bit + i * F.sub_bits, stop = p0 + F.sub_bits;
    uint64_t   st    = huff::pack_state(p0, 0, 0);
    L.se[tid]        = make_uint2((uint32_t)stop, S.end_bit);
    L.ex[tid]        = make_int4(0, 0, 0, 0);
    HUFF_STAMP("start", nsub);
    // a walk of subsequence j from state s (bounds from L.se): its end state and counts into L
    auto walk_sync = [&](int j, uint64_t s0) __attribute__((always_inline)) {
        int              c = (int)(s0 >> 32) & 0xff, k = (int)(s0 >> 40) & 0xff;
        const uint2      se = L.se[j];
        const JpegHuffSeg Sj{0, se.y, 0, 0};
        auto             b   = huff::bits_from(words, Sj, (int)(uint32_t)s0);
        int4             cnt = make_int4(0, 0, 0, 0);
        huff::walk_sync(T, F, b, c, k, (int)se.x, cnt);
        L.en[j] = huff::pack_state(b.p, c, k);
        L.ex[j] = cnt;
    };
    // 1. the guessed start, kHuffLeadBits ahead (the segment's last subsequence ends nobody's start)
    if (have) {
        int4     cnt;
        uint64_t en;
        huff::guess_walk(T, F, S, huff::bits_from(words, S, huff::guess_from(S, p0)), p0, !last, st, en, cnt);
        if (!last) L.en[tid] = en, L.ex[tid] = cnt;
    }
    // 2. Jacobi rounds
    for (int round = 0;; round++) {
        __syncthreads();
        HUFF_STAMP("round", round);
        bool changed = false;
        if (have && !first) {
            const uint64_t e = L.en[tid - 1];
            if (e != st) st = e, changed = true;
        }
        const bool     dirty = changed && !last;
        const uint64_t bal   = __ballot(dirty);
        if (lane == 0) L.wave_n[wave] = __popcll(bal);
        if (!__syncthreads_or(changed)) break;
        int rank = __popcll(bal & ((1ull << lane) - 1)), total = 0;
        for (int w = 0; w < LANES / 64; w++) {
            const int n = L.wave_n[w];
            rank += w < wave ? n : 0;
            total += n;
        }
        if (dirty) L.todo[rank] = tid;
        __syncthreads();
        int      j  = 0;
        uint64_t s0 = 0;
        if (tid < total) j = L.todo[tid], s0 = L.en[j - 1]; // (every start read before any walk writes)
        __syncthreads();
        if (tid < total) walk_sync(j, s0);
    }
    // 3. exclusive prefix (one chunk: nsub <= LANES)
    const int4 cnt = L.ex[tid];
    const int4 s   = wg_scan<LANES>(X, cnt);
    __syncthreads();
    L.ex[tid] = make_int4(s.x - cnt.x, s.y - cnt.y, s.z - cnt.z, s.w - cnt.w);
    __syncthreads();
    HUFF_STAMP("scanned", 0);
    if (!have) return;
    // 4. the final decode
    const int4 e0 = L.ex[S.first_sub], e1 = L.ex[tid];
    const int  per_seg = F.restart * F.bpm, total = F.n_mcu * F.bpm;
    int        c = (int)(st >> 32) & 0xff, k = (int)(st >> 40) & 0xff;
    huff::Out  o;
    o.blk     = sg * per_seg + (e1.x - e0.x) - (k > 0);
    o.blk_end = min(sg * per_seg + per_seg, total);
    o.pred0 = e1.y - e0.y, o.pred1 = e1.z - e0.z, o.pred2 = e1.w - e0.w;
    o.trunc = F.truncated >= 0 && sg >= F.truncated;
    if (o.blk < sg * per_seg) return;
    const int mcu = o.blk / F.bpm;
    o.mx = mcu % F.mcux, o.my = mcu / F.mcux;
    auto b = huff::bits_from(words, S, (int)(uint32_t)st);
    if (!huff::walk_write(T, F, b, c, k, stop, last, o)) atomicOr(error, kJpegCorruptBit);
    HUFF_STAMP("written", b.p - p0);
}

typedef __attribute__((address_space(3))) const uint32_t* lds_words;

// Dynamic LDS (stage_bytes): a copy of the file's data when it fits, so every walk's start and
// refills read LDS instead of device memory.
template <int LANES>
__global__ __launch_bounds__(LANES) void jpeg_huff(const JpegHuffFile* __restrict__ files, int stage_bytes,
                                                   int32_t* __restrict__ error)
{
    __shared__ huff::Tables      T;
    __shared__ Scan              X;
    __shared__ LaneStates<LANES> L;
    extern __shared__ uint32_t   stage[];
    const JpegHuffFile&          F   = files[blockIdx.x];
    const int                    tid = threadIdx.x;
    const bool                   staged = F.nsub <= LANES && F.data_words * 4 <= stage_bytes;

    if (staged) { // 16-byte copies, all in flight before the tables are built
        const auto src = huff::gmem<const uint4>(F.data);
        for (int i = tid; i < (F.data_words + 3) / 4; i += LANES) ((uint4*)stage)[i] = src[i];
    }
#ifdef AEON_HUFF_PROBE
    if (tid == 0) probe_k = 0;
#endif
    HUFF_STAMP("enter", F.data_words);
    huff::tables_codes(T, F, tid, LANES);
    if (tid == 0) X.carry = make_int4(0, 0, 0, 0);
    __syncthreads();
    HUFF_STAMP("codes", 0);
    huff::tables_fast(T, F, tid, LANES);
    huff::tables_long(T, F, tid, LANES);
    __syncthreads();
    HUFF_STAMP("tables", staged);
    if (staged) decode_lanes<LANES>(T, X, L, F, (lds_words)stage, error);
    else if (F.nsub <= LANES) decode_lanes<LANES>(T, X, L, F, huff::gmem<const uint32_t>(F.data), error);
    else decode_strided<LANES>(T, X, F, error);
#ifdef AEON_HUFF_PROBE
    if (blockIdx.x == 0 && tid == 0)
        for (int i = 1; i < probe_k; i++)
            printf("huff %d %d %d\n", i, probe_n[i], (int)(probe_t[i] - probe_t[i - 1]));
#endif
}

// Workgroups of jpeg_huff<LANES> a CU holds at once by its LDS (160 KB on gfx950): one 1,024-lane file,
// two 512-lane ones, three 256-lane ones -- the dynamic part (a file's staged data) is capped to fit.
constexpr int kCuLds = 160 * 1024;
constexpr int huff_files_per_cu(int lanes) { return lanes >= 1024 ? 1 : (lanes >= 512 ? 2 : 3); }

template <int LANES>
int huff_static_lds()
{
    static const int bytes = [] {
        hipFuncAttributes at{};
        return hipFuncGetAttributes(&at, (const void*)jpeg_huff<LANES>) == hipSuccess ? (int)at.sharedSizeBytes : kCuLds;
    }();
    return bytes;
}

// The largest file data (bytes) jpeg_huff<lanes> copies into LDS at its occupancy goal.
int jpeg_huff_stage_cap(int lanes)
{
    const int st = lanes >= 1024 ? huff_static_lds<1024>() : (lanes >= 512 ? huff_static_lds<512>() : huff_static_lds<256>());
    const int cap = (kCuLds / huff_files_per_cu(lanes) - st - 256) & ~15;
    return cap < 0 ? 0 : (cap < kHuffStageMax ? cap : kHuffStageMax);
}

template <int LANES>
hipError_t launch_huff(const JpegHuffFile* files, int n_files, int stage_bytes, int32_t* error, hipStream_t stream)
{
    static const hipError_t a = hipFuncSetAttribute((const void*)jpeg_huff<LANES>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    kHuffStageMax);
    if (a != hipSuccess) return a;
    hipLaunchKernelGGL(jpeg_huff<LANES>, dim3(n_files), dim3(LANES), stage_bytes, stream, files, stage_bytes, error);
    return hipGetLastError();
}

hipError_t launch_jpeg_huff(const JpegHuffFile* files, int n_files, int lanes, int stage_bytes, int32_t* error,
                            hipStream_t stream)
{
    if (n_files <= 0) return hipSuccess;
    stage_bytes = (stage_bytes + 15) & ~15;
    if (lanes == 256) return launch_huff<256>(files, n_files, stage_bytes, error, stream);
    if (lanes == 512) return launch_huff<512>(files, n_files, stage_bytes, error, stream);
    return launch_huff<1024>(files, n_files, stage_bytes, error, stream);
}

} // namespace aeon_hip
