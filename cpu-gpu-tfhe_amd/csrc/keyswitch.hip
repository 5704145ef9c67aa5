// keyswitch.hip — lweKeySwitch on gfx950: three kernels by batch size.
//
// Reference path replaced (gpuParallel/):
//   lweKeySwitch                       lwe-keyswitch-functions.cu:955-987
//   lweKeySwitchTranslate_fromArray    :101-127   (aibar = a_i + 2^15; 8 base-4 digits;
//                                                  result -= ks[i][j][aij] for aij != 0)
//   key layout ks[i][j][h]             lwekeyswitch.cu:3-18 (ks[i][j][0] is a zero sample :919)
// and the reference GPU comparator keySwitch_n_Bit (boot-gates.cu:2425-2479), whose KS
// kernel did 8192 dependent gathers per thread with the b-sum and the accumulator
// round-tripped through the host.
//
//  * k_keyswitch_v5 (the default above the small-batch threshold): the key switch as an exact
//    int8 MFMA product — the 1024 x 8 base-4 digits as a one-hot matrix, the key as four signed
//    byte limbs, v_mfma_i32_32x32x32_i8 tiles, limbs recombined with wrapping shifts;
//  * k_keyswitch_small (<= 12 key switches, and circuit rows): row gathers from the KSK rows
//    [i < 1024][j < 8][h-1 < 3][512] int32 (a row = 500 a + b + pad, 2 KB), split over chunks
//    of key indices with wrapping atomics;
//  * k_keyswitch_v4 (TFHE_AMD_KS5=0): lane = ciphertext, LDS-staged key column blocks.
#include "engine.h"
#include "modarith.h"

#include <algorithm>
#include <cstdlib>

namespace tfhe_amd {

namespace {


// ---------------------------------------------------------------- v4
// Lane = ciphertext.  A workgroup of 4 waves owns 256 ciphertexts and a 4-column slice of
// the output (columns 4 cb .. 4 cb + 3; column 500 is b).  The KSK is repacked per column
// block, [cb][i][j][h = 1..3][4] int32, so a block's slice is one contiguous 384 KB stream;
// chunks of 32 key indices (12 KB) are double-buffered through LDS next to a resident zero
// row (h = 0).  Each lane extracts its own digits (v_bfe) and gathers the 16-B row piece
// with one ds_read_b128 whose base is (i, j)-constant (immediate offset): per (i, j) one
// LDS read, 4 subtracts and 2 VALU of digit/addressing, for 64 ciphertexts at once.
constexpr int kKs4Cols = 4;
constexpr int kKs4Blocks = 126;                 // ceil(501 / 4)
constexpr int kKs4I = 32;                       // key indices per chunk
#ifndef TFHE_AMD_KS4_THREADS
#define TFHE_AMD_KS4_THREADS 256
#endif
constexpr int kKs4Threads = TFHE_AMD_KS4_THREADS;   // = ciphertexts per workgroup
constexpr int kKs4ChunkU4 = kKs4I * kKsT * 3;   // uint4 pieces per chunk = 768
static_assert(kKs4ChunkU4 % kKs4Threads == 0, "chunk must split evenly");
constexpr int kKs4Pieces = kKs4ChunkU4 / kKs4Threads;   // per thread and chunk

// Where lane ct of the key switch reads and writes (gate batches and circuit levels).
struct KsLane {
    const int32_t *ua, *ua2;   // extracted sample(s), kN words each; ua2 may be null
    uint32_t b;                // u_b (+ u2_b) + add_b
    int32_t *ra, *rb;          // result row (kn words) and b word
};
struct KsPlain {               // gate batch: u[ct] (+ u2[ct]) + (0, add_b) -> res[ct]
    const int32_t *u_a, *u_b, *u2_a, *u2_b;
    int32_t add_b;
    int32_t *res_a, *res_b;
    int B;
    __device__ int count() const { return B; }
    __device__ KsLane lane(int ct) const {
        KsLane l;
        l.ua = u_a + (size_t)ct * kN;
        l.ua2 = u2_a ? u2_a + (size_t)ct * kN : nullptr;
        l.b = (uint32_t)u_b[ct] + (uint32_t)add_b + (u2_b ? (uint32_t)u2_b[ct] : 0u);
        l.ra = res_a + (size_t)ct * kn;
        l.rb = res_b + ct;
        return l;
    }
};
struct KsRows {                // circuit level: lane ct = g B + k -> wire ks[g].out, instance k
    const CircKs *ks;
    const int32_t *u_a, *u_b;
    int32_t *wa, *wb;
    int B, nks;
    __device__ int count() const { return B * nks; }
    __device__ KsLane lane(int ct) const {
        const int g = ct / B, k = ct - g * B;
        const CircKs e = ks[g];
        const size_t s1 = (size_t)e.r1 * B + k, so = (size_t)e.out * B + k;
        KsLane l;
        l.ua = u_a + s1 * kN;
        l.b = (uint32_t)u_b[s1] + (uint32_t)e.add_b;
        l.ua2 = nullptr;
        if (e.r2 >= 0) {
            const size_t s2 = (size_t)e.r2 * B + k;
            l.ua2 = u_a + s2 * kN;
            l.b += (uint32_t)u_b[s2];
        }
        l.ra = wa + so * kn;
        l.rb = wb + so;
        return l;
    }
};

// SPLIT > 1: the key indices are split over SPLIT workgroups per (column block, ciphertext
// group), each adds its partial sums into result rows zeroed (and given b) by
// k_keyswitch_small_init: more waves in flight for mid-size batches.
template <class P, int SPLIT>
__global__ __launch_bounds__(kKs4Threads) void k_keyswitch_v4(const uint4 *__restrict__ ksk4, P io) {
    // buf[b][i][j][h][4 cols]: h = 0 is the zero row of lwe-keyswitch-functions.cu:919
    __shared__ __attribute__((aligned(16))) uint4 buf[2][kKs4I * kKsT * 4];   // 2 x 16 KB
    const int part = SPLIT > 1 ? (int)(blockIdx.x % SPLIT) : 0;
    const int bid = SPLIT > 1 ? (int)(blockIdx.x / SPLIT) : (int)blockIdx.x;
    // XCD-aware: workgroups with equal blockIdx % 8 stream the same column blocks
    const int xcd = bid & 7, k = bid >> 3;
    const int cb = (k & 15) * 8 + xcd;
    const int ctg = k >> 4;
    if (cb >= kKs4Blocks) return;                 // whole workgroup: no barrier skipped
    const int tid = threadIdx.x;
    const int ct = ctg * kKs4Threads + tid;
    const bool valid = ct < io.count();
    const KsLane ln = io.lane(valid ? ct : 0);
    for (int t = tid; t < 2 * kKs4I * kKsT; t += kKs4Threads) buf[t >> 8][(t & 255) * 4] = make_uint4(0, 0, 0, 0);

    uint32_t acc[kKs4Cols];
#pragma unroll
    for (int c = 0; c < kKs4Cols; ++c) acc[c] = 0;
    if (SPLIT == 1 && cb * kKs4Cols <= kn && kn < cb * kKs4Cols + kKs4Cols) acc[kn - cb * kKs4Cols] = ln.b;
    constexpr int kIPart = kN / SPLIT;
    const int ibeg = part * kIPart;

    const uint4 *src = ksk4 + ((size_t)cb * kN + ibeg) * kKsT * 3 + tid;
    const uint4 *pa = reinterpret_cast<const uint4 *>(ln.ua + ibeg);
    const uint4 *pa2 = ln.ua2 ? reinterpret_cast<const uint4 *>(ln.ua2 + ibeg) : nullptr;
    // (i, j, h - 1) piece t = tid + threads l of a chunk goes to buf[.][(t / 3) * 4 + t % 3 + 1]
    int dst[kKs4Pieces];
    uint4 p[kKs4Pieces];
#pragma unroll
    for (int l = 0; l < kKs4Pieces; ++l) {
        const int t = tid + kKs4Threads * l;
        dst[l] = (t / 3) * 4 + (t - 3 * (t / 3)) + 1;
    }
    // register prefetch of one chunk: the KSK pieces + this lane's 32 a-values (+ u2's)
#pragma unroll
    for (int l = 0; l < kKs4Pieces; ++l) p[l] = src[kKs4Threads * l];
    uint4 av[kKs4I / 4], av2[kKs4I / 4];
#pragma unroll
    for (int v = 0; v < kKs4I / 4; ++v) {
        av[v] = pa[v];
        av2[v] = pa2 ? pa2[v] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int l = 0; l < kKs4Pieces; ++l) buf[0][dst[l]] = p[l];
    __syncthreads();
    for (int i0 = 0, b = 0; i0 < kIPart; i0 += kKs4I, b ^= 1) {
        uint32_t a[kKs4I];
#pragma unroll
        for (int v = 0; v < kKs4I / 4; ++v) {
            a[4 * v] = av[v].x + av2[v].x + kKsPrecOffset;
            a[4 * v + 1] = av[v].y + av2[v].y + kKsPrecOffset;
            a[4 * v + 2] = av[v].z + av2[v].z + kKsPrecOffset;
            a[4 * v + 3] = av[v].w + av2[v].w + kKsPrecOffset;
        }
        const bool more = i0 + kKs4I < kIPart;
        if (more) {                                          // next chunk, in flight during the gather
            const uint4 *sn = src + (size_t)(i0 + kKs4I) * kKsT * 3;
#pragma unroll
            for (int l = 0; l < kKs4Pieces; ++l) p[l] = sn[kKs4Threads * l];
#pragma unroll
            for (int v = 0; v < kKs4I / 4; ++v) {
                av[v] = pa[(i0 + kKs4I) / 4 + v];
                if (pa2) av2[v] = pa2[(i0 + kKs4I) / 4 + v];
            }
        }
        const uint4 *cur = buf[b];
#pragma unroll
        for (int ii = 0; ii < kKs4I; ++ii) {
            const uint32_t ab = a[ii];
#pragma unroll
            for (int j = 0; j < kKsT; ++j) {
                const uint32_t aij = (ab >> (32 - (j + 1) * kKsBasebit)) & (kKsBase - 1);
                const uint4 r = cur[(ii * kKsT + j) * 4 + (int)aij];
                acc[0] -= r.x; acc[1] -= r.y; acc[2] -= r.z; acc[3] -= r.w;
            }
            // materialise the running sums once per key index: without this LLVM re-associates
            // the 256 subtractions of a chunk into one tree and keeps every gathered row live
            asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
        }
        if (more) {                                          // other buffer: last read one chunk ago
            uint4 *nb = buf[b ^ 1];
#pragma unroll
            for (int l = 0; l < kKs4Pieces; ++l) nb[dst[l]] = p[l];
        }
        __syncthreads();
    }
    if (!valid) return;
#pragma unroll
    for (int c = 0; c < kKs4Cols; ++c) {
        const int col = cb * kKs4Cols + c;
        int32_t *dst = col < kn ? ln.ra + col : col == kn ? ln.rb : nullptr;
        if (!dst) continue;
        if (SPLIT > 1) atomicAdd(reinterpret_cast<unsigned int *>(dst), acc[c]);   // wrapping: exact
        else *dst = (int32_t)acc[c];
    }
}

// ---------------------------------------------------------------- small batches
// ks-v4 streams each 4-column slice of the key through one workgroup per 256 ciphertexts: for
// a handful of ciphertexts that is 126 workgroups running a 32-chunk loop for one live lane
// each (0.16 ms at B = 1).  For small batches the work is spread over key indices instead:
// workgroup (chunk, ct) takes 16 key indices i of ciphertext ct, thread = output column
// (row layout [i][j][h-1][512], column 500 = b), sums its 128 rows (a digit-0 row is loaded
// and multiplied by 0 so that all loads are independent) and adds the partial into the
// result with one 32-bit atomic add (wrapping, so the sum is the exact Torus32 value whatever
// the order); the result rows are zeroed first (k_keyswitch_small_init), lane b gets u_b.
constexpr int kKsSmallChunks = 64;
constexpr int kKsSmallI = kN / kKsSmallChunks;   // 16 key indices per workgroup

template <class P>
__global__ __launch_bounds__(512) void k_keyswitch_small_init(P io) {
    const KsLane ln = io.lane(blockIdx.x);
    const int col = threadIdx.x;
    if (col < kn) ln.ra[col] = 0;
    else if (col == kn) *ln.rb = (int32_t)ln.b;
}

// U = unroll of the key-index loop: fully unrolled (16: all 128 row loads of a thread issued
// together) for the few-ciphertext launches, kKsSmallU once several ciphertexts share the CUs
// (2: B = 16..96 -10..12 % against 4; 1 measured the same as 2, 8 in between)
#ifndef TFHE_AMD_KS_SMALL_U
#define TFHE_AMD_KS_SMALL_U 2
#endif
constexpr int kKsSmallU = TFHE_AMD_KS_SMALL_U;
template <class P, int U>
__global__ __launch_bounds__(512) void k_keyswitch_small(const int32_t *__restrict__ ksk, P io) {
    const int chunk = blockIdx.x, col = threadIdx.x;
    const KsLane ln = io.lane(blockIdx.y);
    if (col > kn) return;
    const int i0 = chunk * kKsSmallI;
    uint32_t acc = 0;
#pragma unroll U
    for (int ii = 0; ii < kKsSmallI; ++ii) {
        const int i = i0 + ii;
        const uint32_t ab = (uint32_t)ln.ua[i] + (ln.ua2 ? (uint32_t)ln.ua2[i] : 0u) + kKsPrecOffset;
        const int32_t *row = ksk + (size_t)i * kKsT * 3 * kKsRow + col;
#pragma unroll
        for (int j = 0; j < kKsT; ++j) {
            const uint32_t h = (ab >> (32 - (j + 1) * kKsBasebit)) & (kKsBase - 1);
            const uint32_t v = (uint32_t)row[(j * 3 + (int)(h ? h : 1u) - 1) * kKsRow];
            acc -= h ? v : 0u;
        }
    }
    int32_t *dst = col < kn ? ln.ra + col : ln.rb;
    atomicAdd(reinterpret_cast<unsigned int *>(dst), acc);
}

// ---------------------------------------------------------------- v5: int8 MFMA product
// The key switch is a product with a one-hot matrix: res = (0, b) - sum_{i, j} KS[i][j][a_ij],
// a_ij = the j-th base-4 digit of u_i + 2^15 (lwe-keyswitch-functions.cu:101-127), is
//   S[m][col] = sum_k A[m][k] W[k][col],  k = (i, j, h),  A[m][k] = [a_ij(m) = h],
//   W[(i, j, h)][col] = KS[i][j][h][col]  (h = 0: the zero row, lwe-keyswitch-functions.cu:919)
// over K = 1024 x 8 x 4 = 32 768.  W is int32; written as 4 balanced signed bytes
// w = sum_b s_b 2^(8 b) mod 2^32 (s_b in [-128, 127]), S = sum_b 2^(8 b) (A W_b) mod 2^32, and
// every A W_b is exact in int32 (|A W_b| <= 8 192 x 128).  So the key switch runs as
// v_mfma_i32_32x32x32_i8 with no rounding anywhere: N = 512 columns (501 used) x 4 limbs,
// interleaved n = 4 col + limb, in 64 N-blocks of 32.
// One K-step (32) = one key index i: lane l (row r = l & 31, half h = l >> 5) gives A bytes
// 16 h + 4 t + hh = [a_{i, 4h+t} = hh], i.e. dword t = 1 << (8 a_{i, 4h+t}); the four digits of a
// lane are one byte x of u_i + 2^15, so the fragment is two 8-B reads of a 16-entry (2-digit) LDS table.
// Its B fragment (16 B at [nb][i][l], pre-arranged by k_ksk_to_v5) is staged per chunk of
// kKs5Ch key indices in LDS and shared by the workgroup's kKs5Waves waves (32 ciphertexts each).
// Operand / result lane maps checked with exact integer data (scripts/mfma_i8_map.hip).
typedef int ks5_v4i __attribute__((ext_vector_type(4)));
typedef int ks5_v16i __attribute__((ext_vector_type(16)));
#ifndef TFHE_AMD_KS5_WAVES
#define TFHE_AMD_KS5_WAVES 8
#endif
constexpr int kKs5Waves = TFHE_AMD_KS5_WAVES;   // M: 8 x 32 = 256 ciphertexts per workgroup
constexpr int kKs5Threads = 64 * kKs5Waves;
constexpr int kKs5Ch = 16;                      // key indices per LDS chunk (16 KB)
constexpr int kKs5Nb = 64;                      // N-blocks: 8 columns x 4 limbs each
constexpr int kKs5Cols = 8 * kKs5Nb;            // 512 >= 501
static_assert(kKs5Cols > kn, "the N-blocks cover every column and b");
constexpr int kKs5ChU4 = kKs5Ch * 64;           // uint4 per chunk
static_assert(kKs5ChU4 % kKs5Threads == 0, "chunk must split evenly");
constexpr int kKs5Pieces = kKs5ChU4 / kKs5Threads;
#ifndef TFHE_AMD_KS5_G
#define TFHE_AMD_KS5_G 8
#endif
constexpr int kKs5G = TFHE_AMD_KS5_G;          // fragment pairs read ahead of their MFMAs

// SPLIT > 1: the key indices are split over SPLIT workgroups per (N-block, M-tile), each adds its
// partial sums (wrapping, exact in any order) into result rows zeroed (and given b) by
// k_keyswitch_small_init — more workgroups for batches that give fewer than 2 per CU.
// MS: 32-ciphertext M-slices per wave sharing each B fragment read (1 or 2).
template <class P, int SPLIT, int MS>
__global__ __launch_bounds__(kKs5Threads) void k_keyswitch_v5(const uint4 *__restrict__ w5, P io) {
    constexpr int kM = 32 * kKs5Waves * MS;           // ciphertexts per workgroup (M-tile)
    constexpr int kG = kKs5G / MS;                     // i-steps per read group
    static_assert(kKs5Ch % kG == 0, "groups split the chunk");
    // one-hot table per 2-digit nibble, one copy per lane of a 32-lane group: lane L reads entry
    // n at [n][L & 31] (8 B), so every ds_read_b64 of a wave is bank-conflict free whatever the
    // digits (a single 256-entry table read with b128 collided on random digits)
    __shared__ __attribute__((aligned(16))) uint2 lut[16][32];
    __shared__ __attribute__((aligned(16))) uint4 bs[2][kKs5Ch][64];
    // digit bytes of the workgroup's ciphertexts for one chunk: dg[buf][half][ct][ii] = bits
    // 24 - 8 half .. 31 - 8 half of u_i + u2_i + 2^15, i = chunk * kKs5Ch + ii
    __shared__ __attribute__((aligned(16))) uint8_t dg[2][2][kM][kKs5Ch];
    // XCD-aware: the M-tiles of one N-block run on one XCD (blockIdx % 8), reading its B stream
    // together through that XCD's L2
    const int bid = (int)blockIdx.x, xcd = bid & 7, kk = bid >> 3;
    const int nb = xcd + 8 * (kk & 7), part = (kk >> 3) % SPLIT, mt = (kk >> 3) / SPLIT;
    constexpr int kChunks = kN / kKs5Ch / SPLIT;   // chunks of this workgroup's key-index range
    const int c0 = part * kChunks;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, r = l & 31, hh = l >> 5;
    for (int e = tid; e < 16 * 32; e += kKs5Threads)
        lut[e >> 5][e & 31] = make_uint2(1u << (8 * ((e >> 7) & 3)), 1u << (8 * ((e >> 5) & 3)));
    // loader role: thread t fetches kPer of the kKs5Ch sample words of ciphertext (t MS) / 2 per
    // chunk (rows past the batch read row 0: their results are never stored, rows are independent)
    constexpr int kPer = kKs5Ch * MS / 2;          // 8 or 16 words: 2 or 4 uint4
    constexpr int kU4 = kPer / 4;
    static_assert(kKs5Threads * kPer == kM * kKs5Ch, "loader mapping");
    const int lct = (tid * MS) >> 1, lpart = MS == 1 ? (tid & 1) : 0;
    const int lg = mt * kM + lct;
    const KsLane lln = io.lane(lg < io.count() ? lg : 0);
    const uint4 *pa = reinterpret_cast<const uint4 *>(lln.ua) + kU4 * lpart;
    const uint4 *pa2 = reinterpret_cast<const uint4 *>(lln.ua2 ? lln.ua2 : lln.ua) + kU4 * lpart;
    const uint32_t m2 = lln.ua2 ? 0xffffffffu : 0u;   // no second sample: add it masked to 0
    pa += c0 * (kKs5Ch / 4);
    pa2 += c0 * (kKs5Ch / 4);
    uint4 uu[kU4], vv[kU4];
#pragma unroll
    for (int q = 0; q < kU4; ++q) {
        uu[q] = pa[q];
        vv[q] = pa2[q];
    }
    auto put_digits = [&](int buf) {
        uint32_t hi[kPer / 4], lo[kPer / 4];   // bytes 3 (half 0) and 2 (half 1) of each word, packed
#pragma unroll
        for (int q = 0; q < kU4; ++q) {
            const uint32_t w[4] = {uu[q].x + (vv[q].x & m2) + kKsPrecOffset, uu[q].y + (vv[q].y & m2) + kKsPrecOffset,
                                   uu[q].z + (vv[q].z & m2) + kKsPrecOffset, uu[q].w + (vv[q].w & m2) + kKsPrecOffset};
            hi[q] = (w[0] >> 24) | ((w[1] >> 24) << 8) | ((w[2] >> 24) << 16) | ((w[3] >> 24) << 24);
            lo[q] = ((w[0] >> 16) & 255u) | (((w[1] >> 16) & 255u) << 8) | (((w[2] >> 16) & 255u) << 16) |
                    (((w[3] >> 16) & 255u) << 24);
        }
        if (kU4 == 2) {
            *reinterpret_cast<uint2 *>(&dg[buf][0][lct][kPer * lpart]) = make_uint2(hi[0], hi[1]);
            *reinterpret_cast<uint2 *>(&dg[buf][1][lct][kPer * lpart]) = make_uint2(lo[0], lo[1]);
        } else {
            *reinterpret_cast<uint4 *>(&dg[buf][0][lct][0]) = make_uint4(hi[0], hi[1], hi[2 % kU4], hi[3 % kU4]);
            *reinterpret_cast<uint4 *>(&dg[buf][1][lct][0]) = make_uint4(lo[0], lo[1], lo[2 % kU4], lo[3 % kU4]);
        }
    };
    const uint4 *src = w5 + ((size_t)nb * kN + (size_t)c0 * kKs5Ch) * 64 + tid;
    uint4 p[kKs5Pieces];
#pragma unroll
    for (int q = 0; q < kKs5Pieces; ++q) p[q] = src[q * kKs5Threads];
#pragma unroll
    for (int q = 0; q < kKs5Pieces; ++q) (&bs[0][0][0])[tid + q * kKs5Threads] = p[q];
    put_digits(0);
    __syncthreads();
    ks5_v16i acc[MS];
#pragma unroll
    for (int m = 0; m < MS; ++m) acc[m] = ks5_v16i{};
    for (int c = 0; c < kChunks; ++c) {
        const bool more = c + 1 < kChunks;
        {   // next chunk in flight during this one (the last iteration reloads its own: harmless)
            const int cn = more ? c + 1 : c;
            const uint4 *sn = src + (size_t)cn * kKs5ChU4;
#pragma unroll
            for (int q = 0; q < kKs5Pieces; ++q) p[q] = sn[q * kKs5Threads];
#pragma unroll
            for (int q = 0; q < kU4; ++q) {
                uu[q] = pa[cn * (kKs5Ch / 4) + q];
                vv[q] = pa2[cn * (kKs5Ch / 4) + q];
            }
        }
        uint32_t xw[MS][4];
#pragma unroll
        for (int m = 0; m < MS; ++m) {
            const uint4 xd = *reinterpret_cast<const uint4 *>(&dg[c & 1][hh][wave * 32 * MS + 32 * m + r][0]);
            xw[m][0] = xd.x; xw[m][1] = xd.y; xw[m][2] = xd.z; xw[m][3] = xd.w;
        }
        const uint4(*cur)[64] = bs[c & 1];
        // fragments read in groups of kG i-steps (all reads of a group issued before its MFMAs)
#pragma unroll
        for (int g = 0; g < kKs5Ch; g += kG) {
            uint4 av[MS][kG], bv[kG];
#pragma unroll
            for (int q = 0; q < kG; ++q) {
                const int ii = g + q;
#pragma unroll
                for (int m = 0; m < MS; ++m) {
                    const uint32_t xb = xw[m][ii >> 2] >> (8 * (ii & 3));   // digits a_{4hh..4hh+3}, high first
                    const uint2 d01 = lut[(xb >> 4) & 15u][r], d23 = lut[xb & 15u][r];
                    av[m][q] = make_uint4(d01.x, d01.y, d23.x, d23.y);
                }
                bv[q] = cur[ii][l];
            }
            __builtin_amdgcn_sched_barrier(0);   // keep the group's reads ahead of its MFMAs
#pragma unroll
            for (int q = 0; q < kG; ++q) {
                const ks5_v4i b = {(int)bv[q].x, (int)bv[q].y, (int)bv[q].z, (int)bv[q].w};
#pragma unroll
                for (int m = 0; m < MS; ++m) {
                    const ks5_v4i a = {(int)av[m][q].x, (int)av[m][q].y, (int)av[m][q].z, (int)av[m][q].w};
                    acc[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[m], 0, 0, 0);
                }
            }
        }
        if (more) {                              // other buffers: every wave finished them a chunk ago
#pragma unroll
            for (int q = 0; q < kKs5Pieces; ++q) (&bs[(c + 1) & 1][0][0])[tid + q * kKs5Threads] = p[q];
            put_digits((c + 1) & 1);
        }
        __syncthreads();
    }
    // limbs -> Torus32: lane l holds column nb * 8 + (l & 31) / 4, limb l & 3, and ciphertext rows
    // (reg & 3) + 8 (reg >> 2) + 4 hh of each 32-row slice; the quad of lanes 4 q .. 4 q + 3 sums
    // its limbs shifted into place (wrapping: exact mod 2^32) and its first lane stores
    const int col = nb * 8 + (r >> 2);
    const uint32_t lsh = 8u * (uint32_t)(l & 3);
#pragma unroll
    for (int m = 0; m < MS; ++m) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            uint32_t v = (uint32_t)acc[m][reg] << lsh;
            v += (uint32_t)__shfl_xor((int)v, 1, 64);
            v += (uint32_t)__shfl_xor((int)v, 2, 64);
            const int ctm = mt * kM + wave * 32 * MS + 32 * m + (reg & 3) + 8 * (reg >> 2) + 4 * hh;
            if ((l & 3) == 0 && ctm < io.count() && col <= kn) {
                const KsLane lm = io.lane(ctm);
                if (SPLIT > 1) atomicAdd(reinterpret_cast<unsigned int *>(col < kn ? lm.ra + col : lm.rb), 0u - v);
                else if (col < kn) lm.ra[col] = (int32_t)(0u - v);
                else *lm.rb = (int32_t)(lm.b - v);
            }
        }
    }
}

// raw KSK [i][j][h - 1][kKsRow] -> v5 B fragments [nb][i][lane][16 B]: byte 4 t + hh of lane l =
// limb (l & 3) of KS[i][4 (l >> 5) + t][hh][nb * 8 + (l & 31) / 4] as a balanced signed byte
// (0 for hh = 0 and for columns > 500)
__global__ __launch_bounds__(256) void k_ksk_to_v5(const int32_t *__restrict__ ksk, uint4 *__restrict__ w5) {
    const size_t total = (size_t)kKs5Nb * kN * 64;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
        const int l = (int)(t & 63);
        const int i = (int)((t >> 6) % kN);
        const int nb = (int)(t / ((size_t)kN * 64));
        const int col = nb * 8 + ((l & 31) >> 2), limb = l & 3, h = l >> 5;
        uint32_t w[4];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
            uint32_t word = 0;
            for (int hh = 1; hh < 4; ++hh) {
                if (col > kn) break;
                uint32_t v = (uint32_t)ksk[(((size_t)i * kKsT + 4 * h + tt) * 3 + (hh - 1)) * kKsRow + col];
                int8_t sb = 0;
                for (int b = 0; b <= limb; ++b) {          // balanced base-256 digits, low first
                    sb = (int8_t)(v & 0xffu);
                    v = (v - (uint32_t)(int32_t)sb) >> 8;
                }
                word |= (uint32_t)(uint8_t)sb << (8 * hh);
            }
            w[tt] = word;
        }
        w5[t] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// packed KSK [i][j][h - 1][kKsRow] -> v4 [cb][i][j][h - 1][4 cols]
__global__ __launch_bounds__(256) void k_ksk_to_v4(const int32_t *__restrict__ ksk, uint4 *__restrict__ ksk4) {
    const size_t pieces = (size_t)kKs4Blocks * kN * kKsT * 3;
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < pieces; t += (size_t)gridDim.x * 256) {
        const int cb = (int)(t / ((size_t)kN * kKsT * 3));
        const size_t row = t % ((size_t)kN * kKsT * 3);
        ksk4[t] = *reinterpret_cast<const uint4 *>(ksk + row * kKsRow + cb * kKs4Cols);
    }
}

}  // namespace

// ks-v4 launch: batches of at most `ks_split_max()` key switches split the key indices over 2
// workgroups (atomic partial sums into zeroed rows) so that more waves are in flight when the
// batch gives fewer than 2 waves per SIMD (B = 128: 0.162 -> 0.093 ms, 256: 0.169 -> 0.102,
// 512: 0.172 -> 0.129, 768: 0.217 -> 0.165)
static int ks_split_max() { return 768; }   // 128..768: -28..-43 %; 1024 / 4096: +1..3 % (measured)
// Key switches above the small-batch range run on the int8 MFMA kernel (ks-v5) whenever the
// context built its key layout, which it does unless TFHE_AMD_KS5=0 (then ks-v4: A/B runs)
bool ks5_enabled() {
    static const bool v = [] {
        const char *e = getenv("TFHE_AMD_KS5");
        return !(e && atoi(e) == 0);
    }();
    return v;
}
// key-index split of ks-v5: enough workgroups for about 2 per CU (512 for 256 CUs) when the
// batch has few M-tiles
static int ks5_split(int mtiles) {
    int sp = 1;
    while (sp < 8 && mtiles * kKs5Nb * sp < 512) sp *= 2;
    return sp;
}
template <class P, int MS>
static void launch_ks5(const uint4 *w5, int count, const P &io, hipStream_t s) {
    const int mtiles = (count + 32 * kKs5Waves * MS - 1) / (32 * kKs5Waves * MS);
    const int split = ks5_split(mtiles);
    if (split > 1) hipLaunchKernelGGL(k_keyswitch_small_init<P>, dim3(count), dim3(512), 0, s, io);
    const dim3 grid(mtiles * kKs5Nb * split);
    trace_kernel(split == 8 ? "k_keyswitch_v5(int8-mfma+split8)" : split == 4 ? "k_keyswitch_v5(int8-mfma+split4)"
                 : split == 2 ? "k_keyswitch_v5(int8-mfma+split2)" : "k_keyswitch_v5(int8-mfma)");
    switch (split) {
    case 8: hipLaunchKernelGGL((k_keyswitch_v5<P, 8, MS>), grid, dim3(kKs5Threads), 0, s, w5, io); break;
    case 4: hipLaunchKernelGGL((k_keyswitch_v5<P, 4, MS>), grid, dim3(kKs5Threads), 0, s, w5, io); break;
    case 2: hipLaunchKernelGGL((k_keyswitch_v5<P, 2, MS>), grid, dim3(kKs5Threads), 0, s, w5, io); break;
    default: hipLaunchKernelGGL((k_keyswitch_v5<P, 1, MS>), grid, dim3(kKs5Threads), 0, s, w5, io); break;
    }
}
template <class P>
static void launch_ks4(const DeviceKey &key, int groups, int count, const P &io, hipStream_t s) {
    if (key.ksk5) {
        const uint4 *w5 = reinterpret_cast<const uint4 *>(key.ksk5);
        // one M-slice per wave: two slices sharing each B-fragment read (MS = 2, 157 VGPRs) measured
        // slower at every batch (B = 1024 0.089 -> 0.128 ms, 4096 0.306 -> 0.399)
        launch_ks5<P, 1>(w5, count, io, s);
        return;
    }
    trace_kernel("k_keyswitch_v4");
    if (count <= ks_split_max()) {
        hipLaunchKernelGGL(k_keyswitch_small_init<P>, dim3(count), dim3(512), 0, s, io);
        hipLaunchKernelGGL((k_keyswitch_v4<P, 2>), dim3(2 * 128 * groups), dim3(kKs4Threads), 0, s,
                           reinterpret_cast<const uint4 *>(key.ksk4), io);
    } else {
        hipLaunchKernelGGL((k_keyswitch_v4<P, 1>), dim3(128 * groups), dim3(kKs4Threads), 0, s,
                           reinterpret_cast<const uint4 *>(key.ksk4), io);
    }
}

// largest key-switch count for the fully unrolled small kernel: B = 1 0.028 -> 0.021 ms; at B = 8
// the 2-way unroll is already faster (0.029 vs 0.031 ms)
static int ks_unroll_max() { return 4; }

// largest key-switch count that takes the small-batch kernels: the crossover with ks-v5 (split 8:
// 0.036 ms flat up to 256) lies between 12 and 16 (B = 16: 0.039 vs 0.036 ms, B = 1: 0.021 vs
// 0.036); with ks-v4 (TFHE_AMD_KS5=0) between 64 and 128
static int ks_small_max() { return ks5_enabled() ? 12 : 96; }

hipError_t launch_keyswitch_rows(const DeviceKey &key, int B, int nks, const CircKs *ks, const int32_t *u_a,
                                 const int32_t *u_b, int32_t *wa, int32_t *wb, hipStream_t s) {
    if (B <= 0 || nks <= 0) return hipSuccess;
    KsRows io{ks, u_a, u_b, wa, wb, B, nks};
    if ((long)B * nks <= ks_small_max()) {
        trace_kernel("k_keyswitch_small");
        hipLaunchKernelGGL(k_keyswitch_small_init<KsRows>, dim3(B * nks), dim3(512), 0, s, io);
        if ((long)B * nks <= ks_unroll_max())
            hipLaunchKernelGGL((k_keyswitch_small<KsRows, kKsSmallI>), dim3(kKsSmallChunks, B * nks), dim3(512), 0, s,
                               key.ksk, io);
        else
            hipLaunchKernelGGL((k_keyswitch_small<KsRows, kKsSmallU>), dim3(kKsSmallChunks, B * nks), dim3(512), 0, s,
                               key.ksk, io);
        return hipGetLastError();
    }
    const int groups = (int)(((size_t)B * nks + kKs4Threads - 1) / kKs4Threads);
    launch_ks4(key, groups, B * nks, io, s);
    return hipGetLastError();
}

// bootstrap-free circuit nodes: W[out] = (0, c) + s W[in]; one thread per (node, instance, word)
__global__ __launch_bounds__(256) void k_circuit_linear(int B, int nlin, const CircLin *__restrict__ lin,
                                                        int32_t *__restrict__ wa, int32_t *__restrict__ wb) {
    const size_t total = (size_t)nlin * B * (kn + 1);
    for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
        const int w = (int)(t % (kn + 1));
        const size_t gk = t / (kn + 1);
        const int g = (int)(gk / B), k = (int)(gk - (size_t)g * B);
        const CircLin e = lin[g];
        const size_t so = (size_t)e.out * B + k, si = (size_t)(e.in < 0 ? 0 : e.in) * B + k;
        if (w < kn) wa[so * kn + w] = e.in < 0 ? 0 : (int32_t)((uint32_t)e.s * (uint32_t)wa[si * kn + w]);
        else wb[so] = (int32_t)((uint32_t)e.c + (e.in < 0 ? 0u : (uint32_t)e.s * (uint32_t)wb[si]));
    }
}

size_t ksk_v4_words() { return (size_t)kKs4Blocks * kN * kKsT * 3 * 4; }
size_t ksk_v5_words() { return (size_t)kKs5Nb * kN * 64 * 4; }

hipError_t launch_ksk_to_v5(const int32_t *d_ksk, int32_t *d_ksk5, hipStream_t s) {
    hipLaunchKernelGGL(k_ksk_to_v5, dim3(4096), dim3(256), 0, s, d_ksk, reinterpret_cast<uint4 *>(d_ksk5));
    return hipGetLastError();
}

// current_variance bookkeeping of B key-switched samples (tfhe_api.cpp tfhe_amd_boots_batch and the
// Tier-1 queue): per sample the reference's sum over i < 1024, j < 8 of the variance of the
// key-switching-key row its non-zero digit selects (lweKeySwitchTranslate_fromArray,
// lwe-keyswitch-functions.cu:101-127; lwe-functions.cu:150), in the same i, j order with the same
// IEEE double adds, so the doubles are the reference's.  One thread per sample (halves = 2: the
// MUX's u1 + u2).  var [1024][8][4], then var[kKsVarUniform] != 0 when every row has the same
// variance (the reference's lweCreateKeySwitchKey encrypts every row with the same alpha): the sum
// of k such adds is then table[k] = var[kKsVarUniform + 1 + k], built on the host in the same order,
// and a sample needs only its count of non-zero digits.
__device__ __forceinline__ double ks_var_one(const int32_t *__restrict__ u, const int32_t *__restrict__ u2,
                                             const double *__restrict__ var) {
    static_assert(kKsT * kKsBasebit == 16 && kKsBase == 4, "digit count below assumes 8 base-4 digits");
    if (var[kKsVarUniform] != 0.0) {
        int k = 0;
#pragma unroll 8
        for (int i = 0; i < kN; ++i) {
            const uint32_t x = ((uint32_t)u[i] + (u2 ? (uint32_t)u2[i] : 0u) + kKsPrecOffset) >> 16;
            k += __builtin_popcount((x | (x >> 1)) & 0x5555u);   // non-zero 2-bit digits
        }
        return var[kKsVarUniform + 1 + k];
    }
    double v = 0.0;
    // 4 coefficients = 32 table reads in flight per round (a one-thread-per-sample sum is a chain
    // of dependent adds; its loads must not be): a zero digit reads entry 0 of its row and adds
    // +0.0, which leaves v (>= +0) unchanged, exactly as skipping it
    constexpr int U = 4;
    for (int i0 = 0; i0 < kN; i0 += U) {
        uint32_t ab[U];
#pragma unroll
        for (int k = 0; k < U; ++k) ab[k] = (uint32_t)u[i0 + k] + (u2 ? (uint32_t)u2[i0 + k] : 0u) + kKsPrecOffset;
        double t[U][kKsT];
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int j = 0; j < kKsT; ++j) {
                const uint32_t aij = (ab[k] >> (32 - (j + 1) * kKsBasebit)) & (uint32_t)(kKsBase - 1);
                t[k][j] = var[((i0 + k) * kKsT + j) * kKsBase + aij];
            }
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int j = 0; j < kKsT; ++j) {
                const uint32_t aij = (ab[k] >> (32 - (j + 1) * kKsBasebit)) & (uint32_t)(kKsBase - 1);
                v = __dadd_rn(v, aij ? t[k][j] : 0.0);
            }
    }
    return v;
}

__global__ __launch_bounds__(64) void k_ks_variance(const int32_t *__restrict__ u_a, int B, int halves,
                                                    const double *__restrict__ var, double *__restrict__ out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= B) return;
    out[g] = ks_var_one(u_a + (size_t)g * kN, halves == 2 ? u_a + ((size_t)B + g) * kN : nullptr, var);
}

// the same for a mixed-kind batch (tfhe_amd_gate_batch_mixed_host): gate g's key-switch input is
// extracted row ks[g].r1 (+ row ks[g].r2 for a MUX)
__global__ __launch_bounds__(64) void k_ks_variance_rows(const int32_t *__restrict__ u_a, int B,
                                                         const CircKs *__restrict__ ks, const double *__restrict__ var,
                                                         double *__restrict__ out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= B) return;
    const CircKs k = ks[g];
    out[g] = ks_var_one(u_a + (size_t)k.r1 * kN, k.r2 >= 0 ? u_a + (size_t)k.r2 * kN : nullptr, var);
}

hipError_t launch_ks_variance_rows(const int32_t *u_a, int B, const CircKs *ks, const double *var, double *out,
                                   hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ks_variance_rows, dim3((B + 63) / 64), dim3(64), 0, s, u_a, B, ks, var, out);
    return hipGetLastError();
}

hipError_t launch_ks_variance(const int32_t *u_a, int B, int halves, const double *var, double *out, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ks_variance, dim3((B + 63) / 64), dim3(64), 0, s, u_a, B, halves, var, out);
    return hipGetLastError();
}

hipError_t launch_circuit_linear(int B, int nlin, const CircLin *lin, int32_t *wa, int32_t *wb, hipStream_t s) {
    if (B <= 0 || nlin <= 0) return hipSuccess;
    const size_t total = (size_t)nlin * B * (kn + 1);
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 65536);
    trace_kernel("k_circuit_linear");
    hipLaunchKernelGGL(k_circuit_linear, dim3(blocks), dim3(256), 0, s, B, nlin, lin, wa, wb);
    return hipGetLastError();
}

hipError_t launch_ksk_to_v4(const int32_t *d_ksk, int32_t *d_ksk4, hipStream_t s) {
    hipLaunchKernelGGL(k_ksk_to_v4, dim3(2048), dim3(256), 0, s, d_ksk, reinterpret_cast<uint4 *>(d_ksk4));
    return hipGetLastError();
}

// key-switch generation for batches above the small-batch range: 5 (int8 MFMA, the default),
// 4 (TFHE_AMD_KS5=0)
int ks_version() { return ks5_enabled() ? 5 : 4; }   // ks-v1 .. v3 were retired in round 4

hipError_t launch_keyswitch(const DeviceKey &key, int B, const int32_t *u_a, const int32_t *u_b,
                            const int32_t *u2_a, const int32_t *u2_b, int32_t add_b,
                            int32_t *res_a, int32_t *res_b, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (B <= ks_small_max()) {
        trace_kernel("k_keyswitch_small");
        KsPlain io{u_a, u_b, u2_a, u2_b, add_b, res_a, res_b, B};
        hipLaunchKernelGGL(k_keyswitch_small_init<KsPlain>, dim3(B), dim3(512), 0, s, io);
        if (B <= ks_unroll_max())
            hipLaunchKernelGGL((k_keyswitch_small<KsPlain, kKsSmallI>), dim3(kKsSmallChunks, B), dim3(512), 0, s,
                               key.ksk, io);
        else
            hipLaunchKernelGGL((k_keyswitch_small<KsPlain, kKsSmallU>), dim3(kKsSmallChunks, B), dim3(512), 0, s,
                               key.ksk, io);
    } else {
        const int groups = (B + kKs4Threads - 1) / kKs4Threads;
        KsPlain io{u_a, u_b, u2_a, u2_b, add_b, res_a, res_b, B};
        launch_ks4(key, groups, B, io, s);
    }
    return hipGetLastError();
}

}  // namespace tfhe_amd
