/*
 * tfhe_amd.h — the batched (Tier-2) C ABI of the MI355X gate-bootstrapping engine.
 *
 * It is the throughput path of SURVEY.md §8(b): the reference's bit-coalesced batch API
 * (LweSample_16 = {int* a [B x n], int* b [B]}, gpuParallel/lwesamples.h:9-13) driven
 * by bootsAND_fullGPU_n_Bit / bootsXOR_fullGPU_n_Bit / bootsMUX_fullGPU_n_Bit
 * (gpuParallel/boot-gates.cu:2845-3024) and bootstrapAndKeySwitch_n_Bit (:2481-2629).
 * Each entry point here replaces one of those; unlike the reference, the `b` halves live
 * on the device too, all gates (incl. NAND/OR/NOR/AND-NY..., which the reference GPU
 * path lacks) are supported, and results are Torus32-exact.
 *
 * Plain pointers and sizes only.  Ciphertext batches are SoA:
 *   a : int32 [B][500] (row stride 500), b : int32 [B]
 * `_dev` functions take DEVICE pointers (resident in HBM) and a hipStream_t passed as
 * void* (NULL = the context's own stream); they enqueue and return (call
 * tfhe_amd_sync to wait).  Successive calls on one context may use different streams: the
 * engine orders the reuse of its scratch between them.  A context serves one host thread at
 * a time (the Tier-1 API gives every calling thread its own lane).  `_host` functions take
 * host pointers and are synchronous.
 * A call makes its context's device current only while it runs: the calling thread's current
 * HIP device (the one torch and hipMalloc use) is the same after the call as before.
 * Every function returns 0 on success or a negative TFHE_AMD_E* code.
 */
#ifndef TFHE_AMD_H
#define TFHE_AMD_H

#include <stdint.h>
#include <stddef.h>
#include "tfhe/tfhe_core.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    TFHE_AMD_OK = 0,
    TFHE_AMD_E_ARG = -1,       /* bad argument / unknown gate / B < 0 */
    TFHE_AMD_E_HIP = -2,       /* a HIP runtime call failed */
    TFHE_AMD_E_NODEVICE = -3,  /* no usable GPU / the HIP kernels are not loadable */
    TFHE_AMD_E_NOMEM = -4
};

/* gate codes (boot-gates.cu:98-448) */
enum {
    TFHE_GATE_NAND = 0, TFHE_GATE_OR = 1, TFHE_GATE_AND = 2, TFHE_GATE_XOR = 3,
    TFHE_GATE_XNOR = 4, TFHE_GATE_NOR = 5, TFHE_GATE_ANDNY = 6, TFHE_GATE_ANDYN = 7,
    TFHE_GATE_ORNY = 8, TFHE_GATE_ORYN = 9, TFHE_GATE_MUX = 10,
    /* circuit-only gates (below): */
    TFHE_GATE_MAJ = 11,    /* majority(a, b, c), one bootstrap */
    TFHE_GATE_XOR3 = 12,   /* a ^ b ^ c, one bootstrap */
    TFHE_GATE_NOT = 13,    /* bootsNOT (boot-gates.cu:242): linear, no bootstrap */
    TFHE_GATE_COPY = 14,   /* bootsCOPY: linear */
    TFHE_GATE_CONST = 15   /* bootsCONSTANT: `a` is the bit value, no inputs */
};

typedef struct TfheAmdContext TfheAmdContext;
typedef struct TfheAmdCircuit TfheAmdCircuit;

/* Device context = the key material of one cloud key on one GPU: the bootstrapping key in
 * the kernels' transform domains (converted on the device from the coefficient-domain key) and the
 * key-switching key, plus a stream and scratch.  Replaces the reference's key upload
 * (gpuParallel/main.cu:165-213 sendBootstrappingKeyToGPUCoalesceExt, :236-254, :364-407). */
int tfhe_amd_context_create(const TFheGateBootstrappingCloudKeySet *bk, int device, TfheAmdContext **out);
/* same from raw arrays: bk int32 [500][4][2][1024], ksk int32 [1024][8][4][501] */
int tfhe_amd_context_create_raw(const int32_t *bk, const int32_t *ksk, int device, TfheAmdContext **out);
int tfhe_amd_context_destroy(TfheAmdContext *ctx);
/* A context on `device` holding a copy of src's converted device key, copied device to device
 * (hipMemcpyPeerAsync: xGMI when the GPUs have peer access, staged by HIP otherwise) instead of a
 * host upload and on-device conversion; the multi-device context builds its slots > 0 this way. */
int tfhe_amd_context_create_replica(TfheAmdContext *src, int device, TfheAmdContext **out);
/* FNV-1a 64 of the context's device key bytes (every domain it holds, in a fixed order) */
int tfhe_amd_context_key_digest(TfheAmdContext *ctx, unsigned long long *digest);
int tfhe_amd_context_device(const TfheAmdContext *ctx);
/* device bytes of the context's key material (the transform-domain bootstrapping keys and the
 * key-switching key layouts its kernels read) */
long long tfhe_amd_context_key_bytes(const TfheAmdContext *ctx);
/* the context's stream as a hipStream_t (void*) */
void *tfhe_amd_context_stream(TfheAmdContext *ctx);
int tfhe_amd_sync(TfheAmdContext *ctx);
/* pre-size the scratch for batches of up to B gates (optional; grows on demand otherwise) */
int tfhe_amd_reserve(TfheAmdContext *ctx, int B);

/* B gates; cc_* only for TFHE_GATE_MUX (result = a ? b : c).  res may alias inputs. */
int tfhe_amd_gate_batch_dev(TfheAmdContext *ctx, int gate, int B,
                            int32_t *res_a, int32_t *res_b,
                            const int32_t *ca_a, const int32_t *ca_b,
                            const int32_t *cb_a, const int32_t *cb_b,
                            const int32_t *cc_a, const int32_t *cc_b, void *stream);
int tfhe_amd_gate_batch_host(TfheAmdContext *ctx, int gate, int B,
                             int32_t *res_a, int32_t *res_b,
                             const int32_t *ca_a, const int32_t *ca_b,
                             const int32_t *cb_a, const int32_t *cb_b,
                             const int32_t *cc_a, const int32_t *cc_b);

/* Caller-owned pinned host buffers (page-locked, portable to every device and mapped into every
 * device's address space at the host address; tfhe_amd_host_alloc checks that and returns NULL
 * otherwise).  When every array of a tfhe_amd_gate_batch_host call lies inside buffers from
 * tfhe_amd_host_alloc, the call skips the library's pinned staging: the blind rotation's gate
 * prologue reads the inputs in place over PCIe (zero-copy, no input copy at all), the key switch
 * writes the results to device memory and one DMA per array copies them straight into the caller's
 * arrays, overlapped with the next slice's blind rotation above one round (the reference's per-gate
 * cudaMemcpy pairs, boot-gates.cu:2489-2615, become one DMA per result array).
 * Only the library's own allocations are recognised, so a freed and reused address is never
 * mistaken for pinned memory.  tfhe_amd_host_free returns TFHE_AMD_E_ARG for a pointer that is not
 * the start of a live buffer; tfhe_amd_host_is_pinned reports whether [p, p + bytes) lies in one. */
void *tfhe_amd_host_alloc(size_t bytes);
int tfhe_amd_host_free(void *p);
int tfhe_amd_host_is_pinned(const void *p, size_t bytes);

/* B gates of MIXED kinds (gates[i] = TFHE_GATE_NAND .. TFHE_GATE_MUX, a host array) in one
 * blind-rotation launch and one key-switch launch (a one-level circuit: a MUX is two rows and a
 * combined key switch); cc_* only read for MUX entries (may be NULL without one).  Host arrays,
 * synchronous; res may alias inputs.  The Tier-1 coalescing queue runs its mixed batches
 * through it. */
int tfhe_amd_gate_batch_mixed_host(TfheAmdContext *ctx, int B, const int *gates,
                                   int32_t *res_a, int32_t *res_b,
                                   const int32_t *ca_a, const int32_t *ca_b,
                                   const int32_t *cb_a, const int32_t *cb_b,
                                   const int32_t *cc_a, const int32_t *cc_b);

/* tfhe_bootstrap_woKS_FFT over B inputs x (n=500) -> u (N=1024): u_a [B][1024], u_b [B] */
int tfhe_amd_bootstrap_woks_batch_dev(TfheAmdContext *ctx, int B, int32_t mu,
                                      const int32_t *x_a, const int32_t *x_b,
                                      int32_t *u_a, int32_t *u_b, void *stream);
/* tfhe_bootstrap_FFT over B inputs (woKS + key switch) */
int tfhe_amd_bootstrap_batch_dev(TfheAmdContext *ctx, int B, int32_t mu,
                                 const int32_t *x_a, const int32_t *x_b,
                                 int32_t *res_a, int32_t *res_b, void *stream);
/* lweKeySwitch over B samples u (N=1024) -> res (n=500) */
int tfhe_amd_keyswitch_batch_dev(TfheAmdContext *ctx, int B,
                                 const int32_t *u_a, const int32_t *u_b,
                                 int32_t *res_a, int32_t *res_b, void *stream);

/* host-pointer (synchronous) versions of the three above */
int tfhe_amd_bootstrap_woks_batch_host(TfheAmdContext *ctx, int B, int32_t mu,
                                       const int32_t *x_a, const int32_t *x_b,
                                       int32_t *u_a, int32_t *u_b);
int tfhe_amd_bootstrap_batch_host(TfheAmdContext *ctx, int B, int32_t mu,
                                  const int32_t *x_a, const int32_t *x_b,
                                  int32_t *res_a, int32_t *res_b);
int tfhe_amd_keyswitch_batch_host(TfheAmdContext *ctx, int B,
                                  const int32_t *u_a, const int32_t *u_b,
                                  int32_t *res_a, int32_t *res_b);

/* Debug/parity entry: run `iters` CMux steps of the blind rotation (i = 0..iters-1,
 * tfhe_MuxRotate_FFT, skipping bara_i == 0 like tfhe_blindRotate_FFT) on B explicit
 * accumulators acc [B][2][1024] in place, with rotations bara [B][iters].  The raw steps of the
 * selected kernel generation, WITHOUT the exactness guard (the fp64 kernel's roundings are not
 * checked): a kernel-test entry.  The exact L1 function is tfhe_blindRotate_FFT (tfhe.h). */
int tfhe_amd_blind_rotate_dev(TfheAmdContext *ctx, int B, int iters, int32_t *acc,
                              const int32_t *bara, void *stream);
/* tGswFFTExternMulToTLwe (tgsw_functions.h:70, tgsw-fft-operations.cu:124-264) on B accumulators:
 * acc [B][2][1024] <- BK_i (x) acc with i = key_index[b] (device arrays), exact (the NTT kernel's
 * arithmetic); the reference replaces the accumulator by the product the same way.  An index
 * outside [0, 500) leaves its accumulator unchanged (checked on the device). */
int tfhe_amd_external_product_dev(TfheAmdContext *ctx, int B, const int32_t *key_index, int32_t *acc,
                                  void *stream);

/* Timing of the engine's own kernels (HIP events on the stream they run on):
 * enable=1 starts accumulating; read returns the summed ms and launch counts of the
 * blind-rotation kernel and the key-switch kernel since enabling. */
int tfhe_amd_profile_enable(TfheAmdContext *ctx, int enable);
int tfhe_amd_profile_read(TfheAmdContext *ctx, double *br_ms, int *br_launches,
                          double *ks_ms, int *ks_launches);

/* ---------------------------------------------------------------- several GPUs
 * A multi-device context holds one replica of the key per device (uploaded and converted on
 * each device concurrently) and one worker thread per device.  A batch of independent gates
 * is split into contiguous shards whose sizes differ by at most one (tfhe_amd_shard_range,
 * the arithmetic of cpu-gpu-tfhe_amd/shard.py); every device runs its shard through the
 * single-device host path and writes disjoint rows of the caller's arrays.  No collective.
 * Generalizes the reference's per-batch chunk loop (gpuParallel/boot-gates.cu:2869-2907) from
 * one GPU to all of them.  `devices` may repeat a device (several contexts on one GPU). */
typedef struct TfheAmdMulti TfheAmdMulti;
int tfhe_amd_multi_create(const TFheGateBootstrappingCloudKeySet *bk, int device_mask, TfheAmdMulti **out);
int tfhe_amd_multi_create_raw(const int32_t *bk, const int32_t *ksk, const int *devices, int ndev,
                              TfheAmdMulti **out);
int tfhe_amd_multi_destroy(TfheAmdMulti *m);
/* the device list (returns its length; fills up to cap entries) */
int tfhe_amd_multi_devices(const TfheAmdMulti *m, int *devices, int cap);
/* the context of device slot i (profiling, guard statistics); owned by the multi-context */
TfheAmdContext *tfhe_amd_multi_context(TfheAmdMulti *m, int i);
/* B gates over the devices, host SoA arrays as tfhe_amd_gate_batch_host; synchronous */
int tfhe_amd_multi_gate_batch_host(TfheAmdMulti *m, int gate, int B, int32_t *res_a, int32_t *res_b,
                                   const int32_t *ca_a, const int32_t *ca_b, const int32_t *cb_a,
                                   const int32_t *cb_b, const int32_t *cc_a, const int32_t *cc_b);
/* Device-resident shards (no PCIe in the loop): slot i's shard of counts[i] gates lives on slot
 * i's device (arrays of per-slot device pointers, SoA as tfhe_amd_gate_batch_dev; cc_* for MUX
 * only, may be NULL otherwise); enqueued on streams[i] (NULL array or entry = the slot context's
 * own stream) and returns without waiting. */
int tfhe_amd_multi_gate_batch_dev(TfheAmdMulti *m, int gate, const int *counts, int32_t *const *res_a,
                                  int32_t *const *res_b, const int32_t *const *ca_a, const int32_t *const *ca_b,
                                  const int32_t *const *cb_a, const int32_t *const *cb_b,
                                  const int32_t *const *cc_a, const int32_t *const *cc_b, void *const *streams);
/* waits for the own stream of every slot context */
int tfhe_amd_multi_sync(TfheAmdMulti *m);
/* A circuit (below) over the devices, device-resident: slot i evaluates counts[i] instances in its
 * own wire arrays [n_wires][counts[i]][500] / [n_wires][counts[i]] (input wires filled); enqueued,
 * returns without waiting. */
int tfhe_amd_multi_circuit_run_dev(TfheAmdMulti *m, TfheAmdCircuit *circ, const int *counts,
                                   int32_t *const *wires_a, int32_t *const *wires_b, void *const *streams);
/* The same from host memory, synchronous: B instances in contiguous shards (tfhe_amd_shard_range);
 * in_a [n_in][B][500], in_b [n_in][B] hold the input wires in_wires[k]; each device copies in its
 * shard, evaluates in its own HBM and copies its shard of the wires out_wires[k] back into
 * out_a [n_out][B][500], out_b [n_out][B].  The reference's matrix-vector product
 * (BOOTS_matrixMultiplication, gpuParallel/main.cu:2342-2462) over every GPU of a node. */
int tfhe_amd_multi_circuit_run_host(TfheAmdMulti *m, TfheAmdCircuit *circ, int B, int n_in, const int *in_wires,
                                    const int32_t *in_a, const int32_t *in_b, int n_out, const int *out_wires,
                                    int32_t *out_a, int32_t *out_b);
/* shard [lo, hi) of `total` gates for rank of world */
int tfhe_amd_shard_range(long long total, int rank, int world, long long *lo, long long *hi);

/* SURVEY.md §8(b) Tier-2 names: tfhe_gpu_init builds (or replaces) the multi-device context of
 * a cloud key over device_mask (bit d = GPU d); tfhe_gpu_boots_batch runs B gates of one kind
 * (TFHE_GATE_*; c_* for MUX only) over it, or over the key's Tier-1 device when no multi-device
 * context was registered.  The context is dropped with the key. */
int tfhe_gpu_init(const TFheGateBootstrappingCloudKeySet *bk, int device_mask);
int tfhe_gpu_boots_batch(int gate, int32_t *res_a, int32_t *res_b, const int32_t *a_a, const int32_t *a_b,
                         const int32_t *b_a, const int32_t *b_b, const int32_t *c_a, const int32_t *c_b, int B,
                         const TFheGateBootstrappingCloudKeySet *bk);

/* Convenience: the same batch over LweSample arrays (Tier-1 structs) with the device
 * context cached per cloud key.  Each sample's a row is gathered straight into pinned staging and
 * each result scattered straight back (slices of 1 024 pipelined); result may be the same array as
 * an input; current_variance is set as the reference's lweKeySwitch sets it (summed on the GPU in
 * the reference's order).  Returns TFHE_AMD_OK or an error code (c may be NULL unless gate = MUX). */
int tfhe_amd_boots_batch(int gate, LweSample *result, const LweSample *a, const LweSample *b,
                         const LweSample *c, int B, const TFheGateBootstrappingCloudKeySet *bk);

/* Number of per-thread lanes (stream + scratch) the Tier-1 API holds for this cloud key;
 * a thread's lanes are released when it exits (0 if the key has no device context). */
int tfhe_amd_tier1_lane_count(const TFheGateBootstrappingCloudKeySet *bk);

/* Concurrent Tier-1 gate calls on one key are coalesced: a calling thread enqueues its gate; a
 * waiting thread that finds one of the queue's two lanes free becomes the leader of the next
 * batch: it waits until every thread inside a gate call and not in a running batch has enqueued
 * (an adaptive window: 200 us at first, then 4x the observed wait + 20 us, within 200 - 1000 us),
 * takes every pending gate and runs them on its lane — one gate kind
 * as one gate batch, several kinds as one mixed launch (one blind rotation + one key switch) per
 * 512 gates — while later calls queue for the next batch, which the other lane can stage and
 * launch while this one is still running (a lone thread runs its gate at once, B = 1).  Results,
 * aliasing and current_variance are as for a lone call.  env TFHE_AMD_TIER1_COALESCE=0 disables
 * the queue (per-thread lanes, B = 1 launches).
 * queue_stats: batches run, gates they held, the largest batch (reset = 1 zeroes them). */
int tfhe_amd_tier1_queue_stats(const TFheGateBootstrappingCloudKeySet *bk, long long *batches, long long *gates,
                               long long *largest, int reset);
/* Where the queue's time went, in ms summed over its batches since the last reset: ms[0] the
 * leaders' straggler waits, [1] packing the requests, [2] the device gate batches (staging, copies,
 * kernels incl. the current_variance sums of single-kind batches, synchronize), [3] the device
 * current_variance sums of mixed-kind batches, [4] unpacking, [5] 0 (reserved). */
int tfhe_amd_tier1_queue_times(const TFheGateBootstrappingCloudKeySet *bk, double ms[6], int reset);
/* Build the key's Tier-1 device context now (HIP initialisation, key upload and conversion on the
 * device, the queue's stream and scratch: 0.1-0.3 s once per process and key) instead of inside
 * the first gate call. */
int tfhe_amd_tier1_prepare(const TFheGateBootstrappingCloudKeySet *bk);

/* Device selection for the Tier-1 (single-gate) API: the GPU used by the cached
 * context of every cloud key (default 0). */
int tfhe_amd_set_default_device(int device);

/* Key material export (host): bk int32 [500][4][2][1024], ksk int32 [1024][8][4][501] */
int tfhe_amd_export_bk(const TFheGateBootstrappingCloudKeySet *bk, int32_t *out);
int tfhe_amd_export_ksk(const TFheGateBootstrappingCloudKeySet *bk, int32_t *out);
/* LWE secret key (int32 [500]) of a secret keyset */
int tfhe_amd_export_lwe_key(const TFheGateBootstrappingSecretKeySet *key, int32_t *out);
/* TLWE secret key (int32 [1024]; k = 1), = the extracted LWE key of woKS outputs */
int tfhe_amd_export_tlwe_key(const TFheGateBootstrappingSecretKeySet *key, int32_t *out);

/* Select the blind-rotation kernel generation: 0 = default (= 6: fp64 FFT external product,
 * the reference's arithmetic, with the exactness guard above), 4 = the exact 2-prime NTT kernel for
 * every launch.  Returns
 * TFHE_AMD_E_ARG for a generation this build lacks.  Process-wide; results are identical. */
int tfhe_amd_select_kernel(int br_version);

/* The kernels (with the variant the launch geometry picked, e.g. "k_blind_rotate_v6(reg-rotation)",
 * "k_blind_rotate_v4(guard)", "k_keyswitch_v5(int8-mfma+split2)") that the context's last batch
 * call enqueued, comma-separated in first-launch order, NUL-terminated into buf[cap].  Returns the
 * full length (which may exceed cap - 1).  For smoke / bench reports of which kernels produced
 * the checked outputs. */
int tfhe_amd_last_kernels(TfheAmdContext *ctx, char *buf, int cap);

/* Exactness guard of the default fp64 FFT blind rotation: every launch checks
 * every rounded external-product coefficient of every ciphertext over its 500 steps against
 * |c - rint(c)| < 1/8 (through the rounding shifter's quarter-ulp bits) and |c| < 2^49; a
 * ciphertext that breaks either (or whose sampled distance reaches a lower threshold set below)
 * is recomputed by the exact 2-prime NTT kernel in the same stream before its key switch.  The rule is statistical, not a proof: a
 * wrong coefficient needs an FFT error >= 1/2, and one that shows a distance < 1/8 needs >= 7/8
 * while all ~10^6 other roundings of that ciphertext stay below 1/8 (real keys: largest
 * distance 0.06-0.08, FFT errors of one step spread over all its coefficients).  guard_stats reads (and optionally resets)
 * the context's largest distance over the sampled coefficients (one per lane and CMux step) and
 * its count of recomputed ciphertexts (it synchronizes the device).  set_guard_threshold is
 * process-wide and can only make the guard stricter: 0 <= distance <= 1/8 (0 recomputes
 * everything: tests), anything else returns TFHE_AMD_E_ARG.  There is no way to turn the guard
 * off. */
int tfhe_amd_guard_stats(TfheAmdContext *ctx, double *max_distance, long long *recomputed, int reset);
int tfhe_amd_set_guard_threshold(double distance);

/* build tag, e.g. "tfhe_amd gfx950 fft64 br-v6 ks-v4" */
const char *tfhe_amd_version(void);

/* Measurement (not on the bootstrapping path): the fp64 FMA rate the device sustains under its
 * power limit, for the roofline in bench.py.  Every SIMD runs `waves_per_simd` waves of
 * independent register-operand v_fma_f64 chains for about `seconds` (<= 30); *tflops = FLOP/s
 * / 1e12 (FMA = 2), *mhz = the shader clock held meanwhile.  0 on success. */
int tfhe_amd_fp64_ceiling(int device, int waves_per_simd, double seconds, double *tflops, double *mhz);

/* ---------------------------------------------------------------- circuits (§8(f) row 1)
 * A circuit is a DAG of gates over SSA wires (ids 0, 1, ... in creation order; every wire
 * is written once).  tfhe_amd_circuit_run_dev evaluates B independent instances: wires are
 * device arrays a [n_wires][B][500], b [n_wires][B] (wire w of instance k at w*B + k), the
 * input wires filled by the caller.  The compiler levels the DAG by bootstrap depth; each
 * level is ONE blind-rotation launch over all of its gates x B instances and ONE key-switch
 * launch (the reference's compound ANDXOR / XORXOR gates, boot-gates.cu:3027-3098, are the
 * two-gate case).  NOT / COPY / CONST cost no bootstrap: they are folded into the gates that
 * read them (and also written to their own wires).
 * Builders return the new wire id (>= 0) or a negative TFHE_AMD_E* code. */
int tfhe_amd_circuit_create(TfheAmdCircuit **out);
int tfhe_amd_circuit_destroy(TfheAmdCircuit *c);
/* number of contexts the circuit holds device state (level tables, scratch) for; a context's
 * state is dropped when the context is destroyed */
int tfhe_amd_circuit_state_count(TfheAmdCircuit *c);
/* `count` fresh input wires; returns the first id */
int tfhe_amd_circuit_inputs(TfheAmdCircuit *c, int count);
/* one gate (TFHE_GATE_*); unused inputs ignored (MUX: a ? b : cc; CONST: a = bit value) */
int tfhe_amd_circuit_gate(TfheAmdCircuit *c, int gate, int a, int b, int cc);
/* a bootstrapped linear combination: sign((0, c0) + sa*a + sb*b + sc*cc) -> {-1/8, +1/8}
 * (b, cc may be -1); the building block of threshold gates */
int tfhe_amd_circuit_lincomb(TfheAmdCircuit *c, int32_t c0, int32_t sa, int a, int32_t sb, int b, int32_t sc,
                             int cc);
/* node w as built: kind 0 input / 1 bootstrapped / 2 linear, gate code (-1 = lincomb),
 * constant, coefficients[3], inputs[3] (for host-side plaintext evaluation in tests) */
int tfhe_amd_circuit_node(const TfheAmdCircuit *c, int w, int *kind, int *gate, int32_t *c0, int32_t *s, int *in);
/* compile (if needed) and report size: wires, gates, bootstraps per instance, depth */
int tfhe_amd_circuit_info(TfheAmdCircuit *c, int *n_wires, int *n_gates, int *n_bootstraps, int *depth);
/* rows (bootstraps) per level, level 0 first (level 0 is bootstrap-free); returns #levels */
int tfhe_amd_circuit_level_sizes(TfheAmdCircuit *c, int *rows_per_level, int cap);
int tfhe_amd_circuit_run_dev(TfheAmdContext *ctx, TfheAmdCircuit *c, int B, int32_t *wires_a, int32_t *wires_b,
                             void *stream);
/* integer builders over little-endian bit vectors of wire ids (Cipher.cpp's layout):
 * ripple-carry add (XOR3 / MAJ full adders, depth nbits; carry_in may be -1) -> carry wire;
 * subtract a - b -> carry wire; parallel-prefix add (depth 2 + log2 nbits) -> carry wire;
 * unsigned multiply nbits x nbits -> 2 nbits (AND partial products, carry-save tree,
 * prefix adder) */
int tfhe_amd_circuit_add(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int carry_in, int *sum);
int tfhe_amd_circuit_sub(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *diff);
int tfhe_amd_circuit_add_prefix(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *sum);
int tfhe_amd_circuit_mul(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *prod);
/* sum_t a_t * b_t over nterms pairs of nbits-bit operands (a, b: nterms * nbits wires, term
 * major) into out_bits bits, mod 2^out_bits: one Dadda tree over all partial products */
int tfhe_amd_circuit_dot(TfheAmdCircuit *c, int nterms, int nbits, const int *a, const int *b, int out_bits,
                         int *out);

/* Cipher's remaining operators (cpuParallel/Cipher.cpp) as level-batched circuits:
 * compare: op 0 a > b, 1 a >= b, 2 a < b, 3 a <= b, 4 a == b, 5 a != b (two's complement when
 *   is_signed; operator> / <= / ==, :597-644) -> the result wire (log-depth trees);
 * minmax: min (want_max = 0, minimum :314-333) or max, one comparison + one MUX level;
 * neg: two's complement (twosComplement :300-311); abs: |a| (absolute :483-505);
 * divu: unsigned restoring division, q = a / b, r = a % b (r nullable; b = 0: q all ones, r = a);
 * div: signed division truncated toward zero (operator/, divInternal, addSign :507-589).
 * All return 0 (or the wire id for compare) or a negative TFHE_AMD_E* code. */
enum { TFHE_AMD_CMP_GT = 0, TFHE_AMD_CMP_GE = 1, TFHE_AMD_CMP_LT = 2, TFHE_AMD_CMP_LE = 3,
       TFHE_AMD_CMP_EQ = 4, TFHE_AMD_CMP_NE = 5 };
int tfhe_amd_circuit_compare(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int op, int is_signed);
int tfhe_amd_circuit_minmax(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int want_max, int is_signed,
                            int *out);
int tfhe_amd_circuit_neg(TfheAmdCircuit *c, int nbits, const int *a, int *out);
int tfhe_amd_circuit_abs(TfheAmdCircuit *c, int nbits, const int *a, int *out);
int tfhe_amd_circuit_divu(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *q, int *r);
int tfhe_amd_circuit_div(TfheAmdCircuit *c, int nbits, const int *a, const int *b, int *q);

#ifdef __cplusplus
}
#endif
#endif
