// ntt_tables.h — modular-arithmetic constants of the exact external product.
//
// The reference evaluates tGswFFTExternMulToTLwe (gpuParallel/tgsw-fft-operations.cu:124-264)
// in a double-precision FFT domain (LagrangeHalfC, fft_processor_fftw.cu:148-204) and
// truncates back to Torus32 (:177).  This engine computes the same sum EXACTLY: a
// negacyclic NTT of length N=1024 modulo two primes q < 2^30 (q == 1 mod 2048), then a
// centred CRT lift and reduction mod 2^32.
//
// Forward transform: Cooley-Tukey with the psi-twist merged in (natural -> bit-reversed);
// inverse: Gentleman-Sande (bit-reversed -> natural).  The 1/N factor and the Montgomery
// factor R = 2^32 of the pointwise MAC are folded into the NTT-domain bootstrapping key.
#pragma once
#include <cstdint>
#include "params.h"

namespace tfhe_amd {

struct NttTables {
    uint32_t psi[2][kN];     // psi^brv(k) mod q (forward twiddle of butterfly group k)
    uint32_t psip[2][kN];    // Shoup companion floor(w * 2^32 / q)
    uint32_t ipsi[2][kN];    // psi^-brv(k) (inverse)
    uint32_t ipsip[2][kN];
    uint32_t ninv[2];        // N^-1 mod q
    uint32_t qinv_neg[2];    // -q^-1 mod 2^32 (Montgomery REDC)
    uint32_t crt_h;          // q0^-1 mod q1
    uint32_t crt_hp;         // its Shoup companion mod q1
    uint32_t bk_scale[2];    // N^-1 * 2^32 mod q: folded into the NTT-domain key
    uint32_t bk_scalep[2];
};

// host: fill the tables (deterministic; primes are fixed in params.h)
void build_ntt_tables(NttTables *t);

// host helpers shared by the key preprocessing
uint32_t host_powmod(uint32_t b, uint64_t e, uint32_t q);

}  // namespace tfhe_amd
