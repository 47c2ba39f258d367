// Host-side launch entry points of the gfx950 kernels.  Plain C++ (pointers +
// hipStream_t), no torch types, so the .hip translation units build without
// torch headers and the binding layer (csrc/ops.cpp) owns all tensor checks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// ---- elementwise.hip
void tds_relu_fwd(const float* x, float* y, int64_t n, hipStream_t st);
void tds_relu_bwd(const float* g, const float* out, float* dx, int64_t n, hipStream_t st);
void tds_maxpool2_fwd(const float* x, float* y, uint8_t* idx, int64_t planes, int H, int W, hipStream_t st);
void tds_maxpool2_bwd(const float* gy, const uint8_t* idx, float* gx, int64_t planes, int H, int W, hipStream_t st);
void tds_upsample_bilinear_u8(const uint8_t* src, void* dst, bool u8_out, int B, int h, int w, int H, int W,
                              hipStream_t st);

#define TDS_SGD_MAX_TENSORS 48
struct SgdChunkTable {
  float* param[TDS_SGD_MAX_TENSORS];
  const float* grad[TDS_SGD_MAX_TENSORS];
  float* mom[TDS_SGD_MAX_TENSORS];
  int64_t numel[TDS_SGD_MAX_TENSORS];
  int n;
};
void tds_sgd_multi(const SgdChunkTable& tab, float lr, float wd, float momentum, float dampening, int nesterov,
                   int first_step, int64_t max_numel, hipStream_t st);
void tds_cross_entropy(const float* logits, const int64_t* labels, float* row_loss, float* dlogits, float* loss,
                       float* inv_count, int M, int N, int64_t ignore_index, float label_smoothing, hipStream_t st);
void tds_scale_by_device_scalar(const float* in, const float* s, float* out, int64_t n, hipStream_t st);

// ---- conv_generic.hip (NCHW fp32, stride 1, square kernel)
int tds_conv2d_fwd_f32(const float* in, const float* w, const float* bias, float* out, int B, int Cin, int Cout, int H,
                       int W, int KS, int P, hipStream_t st);
void tds_conv2d_flip_weights(const float* w, float* wt, int Cout, int Cin, int KS, hipStream_t st);
int64_t tds_conv2d_wgrad_f32(const float* in, const float* g, float* dw, float* db, float* slab, int B, int Cin,
                             int Cout, int H, int W, int KS, int P, float scale, int accumulate, int num_wg,
                             hipStream_t st);

// ---- batchnorm.hip (NCHW fp32)
int tds_bn_num_chunks(int B, int C, int64_t HW);
void tds_bn_fwd_train(const float* x, int B, int C, int64_t HW, float eps, float momentum, const float* gamma,
                      const float* beta, float* save_mean, float* save_invstd, float* running_mean, float* running_var,
                      int64_t* num_batches, float* aff_a, float* aff_b, double* partial, int nchunk, hipStream_t st);
void tds_bn_eval_affine(const float* rm, const float* rv, int C, float eps, const float* gamma, const float* beta,
                        float* aff_a, float* aff_b, hipStream_t st);
void tds_bn_apply(const float* x, const float* aff_a, const float* aff_b, float* y, int B, int C, int64_t HW, int relu,
                  hipStream_t st);
void tds_bn_bwd(const float* dy, const float* x, int B, int C, int64_t HW, const float* gamma, const float* mean,
                const float* invstd, float* dx, float* dgamma, float* dbeta, float* kbuf, double* partial, int nchunk,
                hipStream_t st);

// ---- linear.hip (skinny M<=8, N<=16)
int tds_linear_fwd_nblk(int64_t K);
int tds_linear_dw(const float* dy, const float* x, float* dW, float* db, int M, int N, int64_t K, int64_t ldw,
                  float scale, int acc, float upd_lr, hipStream_t st);
int tds_linear_fwd_skinny(const float* x, const float* W, const float* bias, float* out, float* partial, int M, int N,
                          int64_t K, int nblk, hipStream_t st);
int tds_linear_bwd_skinny(const float* dy, const float* x, const float* W, float* dx, float* dW, float* db, int M,
                          int N, int64_t K, float scale, int acc_w, hipStream_t st);

// ---- launch_status.hip (TDS_LAUNCH_CHECK, common.h)
int tds_take_launch_error(char* buf, int n);  // 1 (and the message) if a launch failed since the last call
void tds_launch_probe(int* out, int lds_bytes, int threads, hipStream_t st);  // test hook: a launch of any config

// ---- conv2_pack.hip / conv2_fwd2.hip / conv2_bwd.hip (NHWC, fp16x2 split MFMA)
// mag (optional): 33 words of magnitude bounds [max|y2| per channel (32) | max|g2m|], zeroed here
// write_p1: store mag[kMagScales + 1] = 1 / p1_scale (1 without p1_scale); false: the layer-1 Gram
// launch stores it (the packing then runs ahead of layer 1 on a side stream)
void tds_conv2_pack_weights(const float* w2, short* wp, short* wd, uint32_t* mag, const float* p1_scale,
                            hipStream_t st, bool write_p1 = true);
int tds_conv2_num_wg();  // CUs (tds_device_cus)
// ---- cu_budget.hip: CUs the persistent kernels may use (all minus a reserve for RCCL) and
// CU-masked compute streams
int tds_device_cus();
void tds_set_cu_reserve(int n);
int tds_cu_reserve();
hipStream_t tds_cu_masked_stream(int device, int reserve, bool striped);
hipStream_t tds_cu_comm_stream(int device);
hipStream_t tds_cu_side_stream(int device, bool comm);  // a further stream on one side of the split
int tds_cu_release_streams();  // destroy every CU-masked stream (end of a run); returns the count
void tds_comm_spin(int64_t us, int nblocks, int lds_bytes, int* sink, hipStream_t st);
void tds_cu_probe(int64_t us, int nblocks, int* out, hipStream_t st);
int tds_tile_order_fill(int* out, int B, int tiles_r, int tiles_c, int group_rows);  // host: blocked tile order table
void tds_conv2_wgrad_reduce(const float* slab, int nwg, float* dw, float* db, float scale, hipStream_t st);
int tds_conv2_fwd2_num_wg();  // BN2 partial rows the forward writes (workgroups it launches)
void tds_conv2_fwd2_tiles(int P, int* tiles_r, int* tiles_c);
// y2h [B,P,P,32] fp16 (conv2_common.h); ya pooled-blocked (pooled_layout.h), max/min of each 2x2
// window of y2 by sign(gamma2); a2 [B][P/2][P/2][2]: the windows' argmax codes (conv2_common.h)
// ypart (optional): max |y2 - b2| per (channel, workgroup), [32][nwg] float bits
// scales (optional): mag + kMagScales (conv2_pack.hip), the packed weights' and p1's inverse scales
// BN finalize inside a producer launch (conv2_fwd2: BN2): parameters and the outputs it writes
struct TdsBnFin {
  const float* beta;
  float eps, momentum;
  float* stats;          // [2C] mean | invstd
  float* running_mean;   // nullable
  float* running_var;
  int64_t* num_batches;  // nullable
  float* aff;            // [2C] a | b
  uint32_t* mag;         // conv2_fwd2: [32] max |y2 - b2| (float bits), nullable
  double* dwork;         // tds_conv2_fwd2_fin_doubles(nwg)
  uint32_t* uwork;       // tds_conv2_fwd2_fin_words(nwg)
};
int tds_conv2_fwd2_fin_doubles(int nwg);
int tds_conv2_fwd2_fin_words(int nwg);
void tds_conv2_fwd2(const void* p1, const short* wp, const float* bias, const float* gamma, void* y2h, unsigned short* ya,
                    uint32_t* a2, double* partial, uint32_t* ypart, const uint32_t* scales, const int* order, int nwg, int sw, int sk,
                    int B, int P, hipStream_t st, const TdsBnFin* bn = nullptr);
int tds_conv2_bwd3_num_wg();  // slab rows the backward writes (workgroups it launches)
void tds_conv2_bwd3_tiles(int P, int* tiles_r, int* tiles_c);
// rolling-window backward (conv2_bwd.hip): walk = tds_conv2_bwd_walk table for nwg workgroups
// mag: the forward's / head backward's magnitude bounds (the fp16 scale of dy2) and the y2h
// decode (conv2_common.h); b2: conv2.bias (y2h is bias-free)
// dp1h [B][P][ceil(P/4)][16][4] fp16 (conv2_common.h); its decode factor goes to mag[kMagScales + 4]
// a2: the forward's pooling argmax codes (conv2_common.h)
void tds_conv2_bwd3(const void* y2h, const uint32_t* a2, const unsigned short* g2m, const float* aff2, const float* kbuf, const float* b2,
                    uint32_t* mag, const void* p1, const short* wd, void* dp1h, float* slab, const int* walk,
                    int nwg, int sw, int sk, int B, int P, hipStream_t st);
// host: per-workgroup tile lists of vertical segments of ~seg tiles; out == nullptr -> length
int64_t tds_conv2_bwd_walk(int* out, int B, int tiles_r, int tiles_c, int nwg, int seg);

// ---- convnet_fused.hip
int tds_fused_num_wg(int per_cu);
void tds_l1_gram(const double* ac_sum, const double* strips, const void* x, bool levels, int B, int H, int W,
                 const float* w1,
                 double* gram, double* sums, const float* b1, float eps, float momentum, const float* gamma,
                 const float* beta, float* stats, float* running_mean, float* running_var, int64_t* num_batches,
                 float* aff, hipStream_t st, uint32_t* p1inv = nullptr);  // Gram + patch sums + the BN1 finalize
// (p1inv: where to store 1 / p1_scale as the conv2 kernels read it, mag + kMagScales + 1, or nullptr)
// levels: x is uint8 levels (x = level / 255, convnet_fused.hip L1_LEVEL_SCALE), else fp32
void tds_l1_apply(const void* x, bool levels, const float* w1, const float* b1, const float* aff, void* p1,
                  uint8_t* idx1, int nwg, int B, int H, int W, hipStream_t st);
void tds_bn_finalize_shifted(const double* partial, int C, int nchunk, int64_t n, const float* shift, float eps,
                             float momentum, const float* gamma, const float* beta, float* stats, float* running_mean,
                             float* running_var, int64_t* num_batches, float* aff, hipStream_t st);
int tds_x_autocorr_num_wg(int B, int H, int W);  // partial rows tds_x_autocorr writes
void tds_x_moments(const float* x, double* ac_partial, int nwg, double* strips, int B, int H, int W, hipStream_t st);
// border = false: the autocorrelation partials only (the strips then come from tds_l1_reduce_gram's border)
void tds_x_moments_u8(const uint8_t* x, double* ac_partial, int nwg, double* strips, int B, int H, int W,
                      hipStream_t st, bool border = true);
// the uint8 levels' border strips alone [B][8][82] (fallback of the in-launch border)
void tds_x_border_u8(const uint8_t* x, double* strips, int B, int H, int W, hipStream_t st);
// fused upsample to uint8 levels + autocorrelation partials (ups_moments.hip): partial rows, 0 = unsupported shape
int tds_ups_moments_rows(int B, int h, int w, int H, int W);
void tds_ups_moments_u8(const uint8_t* src, uint8_t* x, double* partial, int nrows, int B, int h, int w, int H, int W,
                        hipStream_t st);  // the same moments of uint8 levels (exact)
int tds_conv2_bwd_clock_read(uint32_t* host, int n);  // DIAG 13 per-wave barrier clocks (diag builds)
void tds_x_border(const float* x, double* strips, int B, int H, int W, hipStream_t st);  // border strips [B][8][82]
void tds_reduce_partials(const double* in, double* out, int n, int nchunk, int inner, int64_t ostride, int64_t kstride,
                         hipStream_t st);
// + dbfc = scale * sum_b dl (when dbfc); + the magnitude bounds (when mag): mag[c] = max of
// ypart[c][0..nyp), mag[C] = max of gpart[0..ngp) (float bits, unsigned max)
void tds_bn_bwd_finalize2(const double* partial, int C, int nchunk, int64_t n, const float* gamma, const float* stats,
                          float* dgamma, float* dbeta, float* kbuf, const float* dl, int B, int NC, float* dbfc,
                          float scale, const uint32_t* ypart, int nyp, const uint32_t* gpart, int ngp, uint32_t* mag,
                          hipStream_t st);
// BN statistics from per-workgroup partials [C][nchunk][2] reduced and finalized in one launch
void tds_bn_reduce_finalize(const double* partial, int C, int nchunk, int64_t n, const float* shift, float eps,
                            float momentum, const float* gamma, const float* beta, float* stats, float* running_mean,
                            float* running_var, int64_t* num_batches, float* aff, hipStream_t st);
int tds_l1_bwd_rows(int nwg);  // partial rows [rows][16][27] tds_l1_bwd writes
// dp1h: the conv2 backward's (conv2_common.h), dp1_dec: its decode factor (float bits, device)
// the layer-1 backward's finalize inside its launch (replaces tds_reduce_partials + tds_l1_finalize)
int tds_l1_bwd_max_per_cu(bool levels);  // occupancy of the variant (hipOccupancy...)
void tds_l1_bwd(const void* x, bool levels, const void* dp1h, const uint32_t* dp1_dec, const void* p1,
                const uint8_t* idx1, double* partial, int nwg, int B, int H, int W, hipStream_t st);
// the partial reductions fused with the single-workgroup finalizers (false: no sync words)
bool tds_l1_reduce_finalize(const double* part, int rows, double* bwd_sum, const double* gram, int64_t n,
                            const float* w1, const float* b1, const float* gamma1, const float* stats1, float* dw1,
                            float* db1, float* dgamma1, float* dbeta1, float scale, hipStream_t st);
// line chunks of the in-launch border strips: tds_l1_reduce_gram(border) writes strips [B][8][chunks][82]
int tds_xmom_border_chunks(int H, int W);
// border: workgroups of the same launch form the uint8 levels' border strips (xmom_u8.h) first
bool tds_l1_reduce_gram(const double* ac_part, int nchunk, double* ac_sum, double* strips, const void* x,
                        bool levels, int B, int H, int W, const float* w1, double* gram, double* sums, const float* b1,
                        float eps, float momentum, const float* gamma, const float* beta, float* stats,
                        float* running_mean, float* running_var, int64_t* num_batches, float* aff, hipStream_t st,
                        bool border = false, uint32_t* p1inv = nullptr, const float* pack_w2 = nullptr,
                        short* pack_wp = nullptr, short* pack_wd = nullptr, uint32_t* pack_mag = nullptr);
// (pack_w2 given: 64 extra workgroups pack conv2's weights into pack_wp / pack_wd / pack_mag, as
// tds_conv2_pack_weights(write_p1 = false); p1inv must then be given)
void tds_l1_finalize(const double* bwd_sum, const double* gram, int64_t n, const float* w1, const float* b1,
                     const float* gamma1, const float* stats1, float* dw1, float* db1, float* dgamma1, float* dbeta1,
                     float scale, hipStream_t st);

// ---- head_pb.hip (fc head on the pooled-blocked ya / g2m, pooled_layout.h)
int64_t tds_pb_plane(int Q);  // floats per (image, channel) plane
int tds_head_pb_nblk(int Q);  // workgroups per channel
int tds_head_bwd_pb_nblk(int Q);  // the backward's workgroups per channel (its partial / gpart rows)
// in-launch finalizer counters (launch_status.hip; common.h tds_arrive); nullptr: no fused finalize
uint32_t* tds_sync_words(int site, hipStream_t st);
// a zeroed u64 accumulator block per (device, stream, key) of >= n words (launch_status.hip)
unsigned long long* tds_zeroed_u64(int key, size_t n, hipStream_t st);
bool tds_fused_fin_enabled();  // TDS_FUSED_FIN=0: the separate finalize launches

// partial: [32 * nblk + 32][B*NC] doubles; fused_fin: logits finished in the launch (B <= 8).
// labels (optional, int64 [B]): the cross-entropy loss / dlogits / 1/count formed in the same launch
// (head_pb.hip HPFin) -- returns 1 when it did, 0 when the caller must run tds_cross_entropy, < 0 on
// an unsupported shape
// ya: fp16 [B][32][PB] (conv2_fwd2.hip): y2 at each window's argmax = h d + b2[c], d = inv / 2^k
// from the conv2 pack's scales (ysc = mag + kMagScales, 3 words; nullptr: d = 1)
struct TdsYaDec {
  const float* b2;     // [32]
  const uint32_t* ysc;
};
int tds_head_fwd_pb(const unsigned short* ya, TdsYaDec yd, const float* Wfc, const float* bias, const float* aff2, double* partial,
                    double* sums, float* logits, float* xout, int B, int Q, int NC, hipStream_t st,
                    bool fused_fin = true, const int64_t* labels = nullptr, float* dlogits = nullptr,
                    float* loss = nullptr, float* inv_count = nullptr, int c0 = 0, int c1 = 32);
int tds_head_bwd_pb_npass(int B);
// The activation exchange's fc step from the all-gathered pooled inputs (head_pb.hip head_upd_pb_kernel):
// ya_all [nranks][B][32][PB] fp16 (ya_rs elements per rank), rec [nranks][128] (tds_head_pooled_record),
// dl [nranks * B][NC]; mode 0: out = W - lr * scale * dl^T X (out may be W), 1: out = scale * dl^T X,
// 2: out += scale * dl^T X
int tds_head_upd_pb(const unsigned short* ya_all, int64_t ya_rs, const float* rec, int nranks, const float* dl,
                    const float* W, float* out, int B, int Q, int NC, float scale, float lr, int mode, hipStream_t st);
// a rank's record for tds_head_upd_pb: aff2 [64] | ya scale words [3] (ysc nullptr: 1, 1, 1) | 0 | b2 [32] | 0
void tds_head_pooled_record(const float* aff2, const float* b2, const uint32_t* ysc, float* rec, hipStream_t st);
// channels [c0, c1) only (K-chunked fc gradient: each chunk's dW columns can be all-reduced as
// soon as its launch lands; the BN2 partials of the other channels are left untouched)
// gpart (optional): max |g2m| per workgroup (float bits), [32][npass][nblk]
// hf (optional): the BN2 backward finalize inside the launch (one pass, all channels; replaces
// tds_bn_bwd_finalize2 when the conv2 forward reduced mag[0..32) itself)
struct TdsHeadBwdFin {
  uint32_t* cmax;  // [32] scratch
  const float* stats;
  const float* gamma;
  float* dgamma;
  float* dbeta;
  float* kbuf;     // [96]
  float* dbfc;     // [NC] or nullptr
  uint32_t* mag;   // mag[32] <- max |g2m|, or nullptr
};
// g2m: fp16 [B][32][Q][Q] at a per-channel power-of-two scale 2^e_c (g2inv[c] <- 2^-e_c), bounded
// by the max |W| per channel and class that the last head forward on this stream measured
int tds_head_bwd_pb(const unsigned short* ya, TdsYaDec yd, const float* Wfc, const float* aff2, const float* dlogits, unsigned short* g2m,
                    double* partial, float* dW, float* Wupd, int B, int Q, int NC, float scale, float lr, int c0,
                    int c1, uint32_t* gpart, float* g2inv, hipStream_t st, const TdsHeadBwdFin* hf = nullptr);

// ---- zs_exchange.hip (zero-suppressed fc-input rows, parallel/zs.py)
int64_t tds_zs_npages(int64_t n);
// meta [npages * 65] (offsets + mask words), counts [npages] scratch, vals [cap] (dropped past
// cap), nnz: int64 device scalar
void tds_zs_encode(const float* x, int64_t n, int* meta, float* vals, int64_t cap, int64_t* nnz, hipStream_t st);

void tds_zs_decode(const int* meta, const float* vals, int64_t cap, float* out, int64_t n, hipStream_t st);
// linear_dw with X given as W source ranks' zero-suppressed encodings (decoded in registers)
int tds_linear_dw_zs(const float* dy, const int* meta, int64_t mstride, const float* vals, int64_t cap, int rows,
                     int M, int N, int64_t K, float* dW, int64_t ldw, float* db, float scale, int acc, float upd_lr,
                     hipStream_t st);
// segmented form (the sharded exchange): page table (start, cnt, seg) + per-segment first page /
// page count; values in fixed-capacity slots per segment; seg_nnz [nseg] int64
void tds_zs_seg_encode(const float* x, const int64_t* pg_start, const int* pg_cnt, const int* pg_seg, int64_t npages,
                       const int* seg_first, const int* seg_npg, int nseg, int* meta, int* counts, float* vals,
                       int64_t cap, int64_t* seg_nnz, hipStream_t st);
void tds_zs_seg_decode(const int* meta, const int64_t* pg_start, const int* pg_cnt, const int* pg_seg, int64_t npages,
                       const float* vals, int64_t cap, float* out, hipStream_t st);
