// params.h — the default gate-bootstrapping parameter set, fixed at compile time.
// new_default_gate_bootstrapping_parameters (gpuParallel/tfhe_gate_bootstrapping.cu:25-49),
// TGswParams ctor (tgsw.cu:7-29), key-switch layout (lwekeyswitch.cu:3-18).
#pragma once
#include <cstdint>

namespace tfhe_amd {

constexpr int kN = 1024;          // ring degree (TLWE N)
constexpr int kLogN = 10;
constexpr int k2N = 2 * kN;
constexpr int kn = 500;           // LWE dimension (in/out)
constexpr int kK = 1;             // TLWE mask polynomials
constexpr int kL = 2;             // gadget decomposition length
constexpr int kBgbit = 10;        // log2 Bg
constexpr int kKpl = (kK + 1) * kL;   // 4 TGSW rows
constexpr int kKsT = 8;           // key-switch digits
constexpr int kKsBasebit = 2;     // key-switch base 4
constexpr int kKsBase = 1 << kKsBasebit;
constexpr uint32_t kDecompOffset = 512u * ((1u << 22) + (1u << 12));   // 2149580800
constexpr uint32_t kKsPrecOffset = 1u << (32 - (1 + kKsBasebit * kKsT)); // 2^15
// current_variance tables (k_ks_variance): the KSK row variances [kN][kKsT][kKsBase], then a flag
// (non-zero: every row has the same variance), then the sequential sums of k copies, k <= kN kKsT
constexpr int kKsVarUniform = kN * kKsT * kKsBase;
constexpr int kKsVarWords = kKsVarUniform + 1 + kN * kKsT + 1;

// Device key-switch key rows: for each (i<1024, j<8) the three non-zero digits h=1..3,
// each row = 500 a-coefficients, b, zero padding to 512 int32 (2 KB, 16-B aligned).
constexpr int kKsRow = 512;

// The exact external product: 2-prime CRT NTT, q < 2^27, q == 1 mod 2N (the two largest
// such primes).  q0*q1 = 1.99976 * 2^53 > 2 * (4 rows * 1024 * 512 * 2^31) = 2^53, so the
// centred CRT lift is exact (SURVEY.md §7.3 option (i)).  q < 2^27 leaves 32q of headroom
// in 32-bit lanes: the lazy forward NTT needs no reductions at all (values stay < 22q).
constexpr uint32_t kQ[2] = {134215681u, 134203393u};

// standard deviations, tfhe_gate_bootstrapping.cu:36-38 (mulBySqrtTwoOverPi :22)
constexpr double kKsStdev = 2.4349504419032758e-05;   // sqrt(2/pi) * 2^-15
constexpr double kBkStdev = 7.180961047225788e-09;    // sqrt(2/pi) * 9e-9
constexpr double kMaxStdev = 0.012466946262544772;    // sqrt(2/pi) * 2^-4 / 4

}  // namespace tfhe_amd
