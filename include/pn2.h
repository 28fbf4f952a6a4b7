/*
 * pn2.h -- C ABI of libpn2.so, the MI355X (gfx950) PointNet++ set-abstraction path.
 *
 * Every entry point:
 *   - takes plain pointers to caller-allocated DEVICE buffers (the caller's allocator owns all
 *     memory; nothing here allocates), element strides as int64, and a hipStream_t passed as
 *     void*;
 *   - is asynchronous on that stream and never synchronises the device, so it may be captured
 *     into a hipGraph;
 *   - returns PN2_OK (0) or a negative PN2_E* code; the message of the last failure on the
 *     calling thread is returned by pn2_last_error() (thread-local).
 *   - is re-entrant across host threads, as the reference's concurrent-inference demo
 *     /root/reference/mutilthreading/predict_test.py:44-63 requires: besides the caller's
 *     buffers the library holds only thread-local state (the error message, a thread's tuning
 *     copy, a thread's device error slots), the process-wide tuning keys (one atomic word per
 *     key) and the process-wide default error slot (kernels only OR into it; its reads are
 *     serialised).
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   pn2_fps_f32            farthest_point_sample            model/pointnet2_utils.py:47-68
 *   pn2_fps_ws_f32         the same, any N (workspace)       model/pointnet2_utils.py:47-68
 *   pn2_fps_host_ws_f32    the same, start drawn on the host model/pointnet2_utils.py:59
 *   pn2_ball_query_multi_i32  query_ball_point per MSG radius   model/pointnet2_utils.py:197-203
 *                          (+ index_points(points, fps_idx)  model/pointnet2_utils.py:106)
 *   pn2_ball_query_f32     query_ball_point + square_distance model/pointnet2_utils.py:70-90, 5-26
 *   pn2_pack_points_f32    torch.sum(points**2,-1) of square_distance model/pointnet2_utils.py:24-25
 *   pn2_square_distance_f32 square_distance                  model/pointnet2_utils.py:5-26
 *   pn2_index_points_f32   index_points                      model/pointnet2_utils.py:28-45
 *   pn2_group_f32          grouping of sample_and_group /    model/pointnet2_utils.py:107-116,
 *                          PointNetSetAbstractionMsg         model/pointnet2_utils.py:204-209
 *   pn2_pack_layer_f32     Conv2d(1x1)+BatchNorm2d(eval) params of the shared MLP
 *                                                            model/pointnet2_utils.py:150-156, 184-193
 *   pn2_sa_mlp_max_f32     grouped shared MLP (conv+bn+relu)* + max over the neighbourhood
 *                                                            model/pointnet2_utils.py:167-172, 211-218
 *   pn2_bn_train_stats_f32 / pn2_bn_relu_apply_f32 (/ pn2_bn_train_forward_f32: both) /
 *   pn2_group_max_f32 / pn2_bn_relu_backward_f32
 *                          train-mode BatchNorm2d + ReLU + torch.max over K, forward and backward
 *                                                            model/pointnet2_utils.py:167-172, 211-221
 *                                                            (under autograd: train_rotation.py:99-133)
 *                          and the v1 shared MLPs' Conv1d + BatchNorm1d (+ ReLU) + max over N
 *                                                            model/pointnet_utils.py:31-35, 118-128
 *   pn2_linear_rows_f32    eval Linear + BatchNorm1d (folded on the host) + ReLU of the FC tails
 *                                                            model/pointnet_utils.py:33-40;
 *                                                            pointnet_cls.py:26-28; rotation.py:45-49;
 *                                                            pointnet2_cls_ssg.py:32-34
 *   pn2_prepare_points_f64 the scripts' input preparation: provider.normalization + torch.Tensor
 *                          + provider.splice_torch + transpose (+ the translation heads' mean)
 *                                                            provider.py:5-21, 166-180;
 *                                                            test_translation.py:72-79
 */
#ifndef PN2_H
#define PN2_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PN2_OK 0
#define PN2_EINVAL (-1)     /* bad argument / shape */
#define PN2_EUNSUPPORTED (-2) /* shape outside what the kernels are built for */
#define PN2_EHIP (-3)       /* HIP runtime error at launch */

#define PN2_ABI_VERSION 17

int pn2_abi_version(void);
const char *pn2_last_error(void);

/* Device error slots: conditions under which the reference raises but a kernel cannot.  The
 * kernels stay in bounds (clamped or NaN outputs, documented per entry point) and OR a bit into
 * the device error slot of the host thread that launched them:
 *   PN2_DEVERR_NO_NEIGHBOUR  a ball-query centroid had no point within the radius (its row is
 *                            padded with N, pointnet2_utils.py:85-89; the reference's next
 *                            index_points raises IndexError); the SA kernels read point 0 there
 *   PN2_DEVERR_INDEX         pn2_index_points_f32 / pn2_group_f32 got an index outside [-N, N)
 *                            (the element is NaN)
 * A launch raises into the slot of the device its STREAM belongs to (hipStreamGetDevice; the
 * current device for the null stream), whatever the thread's current device is.
 * pn2_error_slot_set(slot): from now on, launches by the calling thread on the current device
 * raise into `slot` -- two caller-owned, zeroed uint32 DEVICE words ([0] the bits, [1] scratch
 * for the take) that must outlive every launch and captured graph that uses them (a graph
 * raises into the slot of the thread that captured it).  NULL: back to the process-wide
 * default slot, which every thread without a slot of its own shares.
 * pn2_error_slot_take: the calling thread's slot on `stream`'s device, taken -- read and,
 * when `clear` != 0, reset in ONE device atomic, so a bit raised meanwhile is never lost --
 * stream-ordered on `stream`, which it then waits for.
 * pn2_device_errors: the same take after hipDeviceSynchronize (every stream's work done).
 * pn2.check_device_errors() gives each (thread, device) its own slot and raises IndexError. */
#define PN2_DEVERR_NO_NEIGHBOUR 1u
#define PN2_DEVERR_INDEX 2u
int pn2_error_slot_set(uint32_t *slot);
int pn2_error_slot_take(int clear, uint32_t *bits, void *stream);
int pn2_device_errors(int clear, uint32_t *bits);

/* Kernel-selection tuning: int64 parameters of the launch choices (which kernel family, tile
 * widths, block shapes).  The defaults are the measured best (pn2_tuning_default) and the
 * library never reads the environment; tests and A/B tools change them (pn2/tuning.py applies
 * the one PN2_TUNING="key=value,..." variable at load).  Process-wide keys are atomic words:
 * a set on one thread while another launches is safe (the launch sees the old or the new value
 * of each key).  Keys: pn2_tuning_keys() (space-separated). */
int pn2_tuning_get(const char *key, int64_t *value);
int pn2_tuning_set(const char *key, int64_t value);
int pn2_tuning_default(const char *key, int64_t *value);
const char *pn2_tuning_keys(void);
/* pn2_tuning_local(1): this host thread gets its own copy of the keys (taken from the
 * process-wide values at the outermost enter); pn2_tuning_get/set and every launch on this
 * thread then use the copy, other threads are unaffected; pn2_tuning_local(0) leaves (nested
 * enters count).  pn2.pipeline captures its graphs in this mode under its own launch profile. */
int pn2_tuning_local(int enter);

/* Packed point layout used by the ball query: [B][N][cp] float32, cp = pn2_packed_stride(C),
 * holding the C coordinates, then ssq = torch.sum(p**2,-1) computed with the reference's
 * layout-dependent CPU summation order, then zero padding. */
int64_t pn2_packed_stride(int64_t C);

/* Farthest point sampling over points[b, n, c] = pts[b*sb + n*sn + c*sc].
 * start[B] (int64, device) = the reference's torch.randint draw.  Outputs (device):
 *   out_idx    [B,S] int64                      fps indices
 *   out_pts    [B,S,C] float32 contiguous, or NULL   index_points(points, fps_idx)
 *   out_packed [B,S,cp] float32, or NULL         packed centroids (contiguous-layout ssq)
 *   pts_packed [B,N,cp] float32, or NULL         packed input points (input-layout ssq)
 * C <= 64 (else PN2_EUNSUPPORTED: the reference's channel-sum orders are pinned to C = 64);
 * 16 < C <= 64 always runs the streamed kernel (256 threads per cloud; the same workspace rule
 * with the LDS holding up to 40896 distances).  The cloud is register-resident up to N = 16384 for C == 3, 8192 for
 * C == 10, 4096 for other C (past that, up to N = 16384, the channels after xyz are re-read
 * from pts each iteration unless they are constant over the cloud: one-hot), with S <= 8192.
 * Any other N or S runs the streamed kernel: the points re-read every iteration, the running
 * distances in LDS up to N = 40896, past that in a caller workspace of
 * pn2_fps_workspace_bytes(B, N, C, S) bytes (pn2_fps_ws_f32; pn2_fps_f32 passes none and
 * fails with PN2_EINVAL when one is needed). */
int pn2_fps_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                int64_t sc, const int64_t *start, int64_t S, int64_t *out_idx, float *out_pts,
                float *out_packed, float *pts_packed, void *stream);
int64_t pn2_fps_workspace_bytes(int64_t B, int64_t N, int64_t C, int64_t S);
int pn2_fps_ws_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                   int64_t sc, const int64_t *start, int64_t S, int64_t *out_idx, float *out_pts,
                   float *out_packed, float *pts_packed, void *workspace, int64_t workspace_bytes,
                   void *stream);
/* The same with start_host[B] in HOST memory, as the reference draws it (pointnet2_utils.py:59:
 * torch.randint on the CPU, then .to(device)): read during the call -- the caller may reuse it
 * on return -- and checked (0 <= start < N, else PN2_EINVAL), no host->device copy. */
int pn2_fps_host_ws_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                        int64_t sc, const int64_t *start_host, int64_t S, int64_t *out_idx,
                        float *out_pts, float *out_packed, float *pts_packed, void *workspace,
                        int64_t workspace_bytes, void *stream);

/* Pack a [B,N,C] strided view into [B,N,cp] with its ssq (see above).  C <= 64, as for the
 * ball query and square_distance below (else PN2_EUNSUPPORTED). */
int pn2_pack_points_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                        int64_t sn, int64_t sc, float *packed, void *stream);

/* query_ball_point: for every centroid, the first K point indices (ascending) whose
 * square_distance is not > (float)(radius*radius), padded with the first hit (N if none).
 * pts_packed [B,N,cp], ctr_packed [B,S,cp] from pn2_pack_points_f32 / pn2_fps_f32.
 * out_idx [B,S,K] int64.  Any 1 <= K <= N (rows that fit a 96 KB LDS buffer are built there and
 * written out whole; longer ones are written in place).  K > N is rejected with PN2_EINVAL
 * (the reference raises IndexError).  16 < C <= 64: a register-light kernel that walks the
 * records in index order per centroid (same results; not tuned -- no BASELINE config has it). */
int pn2_ball_query_f32(const float *pts_packed, const float *ctr_packed, int64_t B, int64_t N,
                       int64_t S, int64_t C, double radius, int64_t K, int64_t *out_idx,
                       void *stream);
/* The same, also writing out_cnt [B,S] int32 (or NULL): the number of distinct neighbours of
 * each centroid, min(hits, K) -- out_idx entries past it repeat entry 0.  Passed to the SA MLP
 * (pn2_sa_src.cnt) it lets the chain compute only those rows (the max over a group does not
 * change without repeats). */
int pn2_ball_query_cnt_f32(const float *pts_packed, const float *ctr_packed, int64_t B,
                           int64_t N, int64_t S, int64_t C, double radius, int64_t K,
                           int64_t *out_idx, int32_t *out_cnt, void *stream);
/* The same lists as int32 (half the bytes; the SA layers' fused path reads them through
 * pn2_sa_src.idx32).  Entries, padding and counts as pn2_ball_query_cnt_f32. */
int pn2_ball_query_i32(const float *pts_packed, const float *ctr_packed, int64_t B, int64_t N,
                       int64_t S, int64_t C, double radius, int64_t K, int32_t *out_idx,
                       int32_t *out_cnt, void *stream);
/* nr (1..3) radii of one centroid set in one launch -- the scales of an MSG layer
 * (pointnet2_utils.py:197-203 calls query_ball_point once per radius): each pair's distance
 * computed once and tested against every radius; out_idx[r] [B,S,K[r]] int32 and out_cnt[r]
 * [B,S] (or out_cnt / out_cnt[r] NULL) exactly as nr pn2_ball_query_i32 calls would write them. */
int pn2_ball_query_multi_i32(const float *pts_packed, const float *ctr_packed, int64_t B,
                             int64_t N, int64_t S, int64_t C, int nr, const double *radii,
                             const int64_t *K, int32_t *const *out_idx, int32_t *const *out_cnt,
                             void *stream);

/* square_distance(src, dst) -> out [B,S,N] float32 from packed records of src [B,S,cp] and
 * dst [B,N,cp] (same float32 recipe as the ball query). */
int pn2_square_distance_f32(const float *src_packed, const float *dst_packed, int64_t B,
                            int64_t S, int64_t N, int64_t C, float *out, void *stream);

/* out[b, m, :] = pts[b, idx[b*M + m], :] ; out contiguous [B,M,C]. idx int64 [B,M]. */
int pn2_index_points_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                         int64_t sn, int64_t sc, const int64_t *idx, int64_t M, float *out,
                         void *stream);

/* Grouping: out[b,s,k,:] (contiguous [B,S,K,C+D]) =
 *   feature_first == 0 : [pts[b,idx]-ctr[b,s], feat[b,idx]]   (sample_and_group, SSG)
 *   feature_first == 1 : [feat[b,idx], pts[b,idx]-ctr[b,s]]   (PointNetSetAbstractionMsg)
 * feat may be NULL (D = 0).  ctr is contiguous [B,S,C]; feat element (b,n,d) at
 * feat[b*fb + n*fn + d*fd]. */
int pn2_group_f32(const float *pts, int64_t B, int64_t N, int64_t C, int64_t sb, int64_t sn,
                  int64_t sc, const float *feat, int64_t D, int64_t fb, int64_t fn, int64_t fd,
                  const float *ctr, int64_t S, const int64_t *idx, int64_t K, int feature_first,
                  float *out, void *stream);

/* One shared-MLP layer packed for the kernels: wt = W^T pair-interleaved, [cin_pad/2][cout][2]
 * (element (k, o) at ((k>>1)*cout + o)*2 + (k&1), zero rows past cin), alpha[cout], beta[cout]
 * such that layer(x) = relu(alpha * (W x) + beta): the eval-mode BatchNorm2d folded with the
 * conv bias.  The kernels lay a row out as [features | xyz]; `rot` is the number of leading
 * input channels of W that are xyz (C for sample_and_group / group_all first layers, whose
 * reference order is [xyz, features]; 0 otherwise): row k of wt is input channel (k+rot)%cin.
 * cin_pad = pn2_layer_cin_pad(cin). */
int64_t pn2_layer_cin_pad(int64_t cin);
int pn2_pack_layer_f32(const float *W, const float *bias, const float *gamma, const float *beta,
                       const float *mean, const float *var, double eps, int64_t cout,
                       int64_t cin, int64_t rot, float *wt, float *alpha, float *beta_out,
                       void *stream);

/* Source of the MLP's input rows. */
#define PN2_SRC_GROUP_XYZ_FIRST 0  /* sample_and_group:  [xyz-ctr, feat] rows of group idx   */
#define PN2_SRC_GROUP_FEAT_FIRST 1 /* MSG:               [feat, xyz-ctr] rows of group idx   */
#define PN2_SRC_GROUP_ALL 2        /* sample_and_group_all: [xyz (raw), feat] of every point */
#define PN2_SRC_ROWS 3             /* a dense [M][cin] float32 matrix (row stride rs)        */

typedef struct pn2_mlp_layer {
    const float *wt;    /* [cin_pad][cout] */
    const float *alpha; /* [cout] */
    const float *beta;  /* [cout] */
    int64_t cin;
    int64_t cout;
    const void *wt_split; /* pn2_pack_layer_split_bf16 image of the same W, or NULL */
    int64_t flags;        /* PN2_LAYER_* bits, 0 = the SA layers' conv + BN + ReLU       */
} pn2_mlp_layer;

/* Layer without the ReLU: out = alpha * (W x) + beta (PointNetEncoder's conv3 + bn3 before its
 * max, /root/reference/model/pointnet_utils.py:125-127).  Served by the split dense-layer
 * kernels only (group_all / rows sources); other kernels reject it with PN2_EUNSUPPORTED.  The
 * training entry points (pn2_bn_relu_apply_f32 / pn2_bn_relu_backward_f32) take it as their
 * flags argument. */
#define PN2_LAYER_NO_RELU 1

/* The same W packed for the split chain / dense kernels.  Planes 0-2: three bf16 planes (hi, mid,
 * lo with W = hi + mid + lo to 2^-24 relative), each [cout/32][kblocks][64 lanes][8] in MFMA
 * fragment order; planes 3-4: two fp16 planes (hi, lo) of W[o][.] * 2^e_o in the same order,
 * e_o putting output row o's largest |w| in [2^14, 2^15) (W*2^e = hi + lo to 2^-22 relative);
 * then float [cout] = 2^-e_o.  Kernel input channel k (block k/16) maps to W's input channel as
 * follows:
 *   xyz == 0 (hidden layers): k.   xyz > 0 (first layer, rows [xyz | features], D = cin-xyz):
 *   block 0 holds the xyz channels (k < xyz), blocks >= 1 the features (k-16 < D); W's own
 *   order is [xyz, features] if xyz_first (sample_and_group) else [features, xyz] (MSG).
 * Lane 32h + r, element j of fragment (t, kb) holds W[32t + r][in(16kb + (j&3) + 8(j>>2) + 4h)]
 * (0 for padding).  kblocks = pn2_layer_split_kblocks(cin, xyz); the image takes
 * pn2_layer_split_bytes(cout, cin, xyz) bytes, 16-byte aligned.  Chains given wt_split for
 * every layer (3 layers, grouped rows, hidden widths 32..128) run as one register-resident
 * kernel with fp32-accurate arithmetic: split fp16 (3 MFMAs per product, both operands scaled
 * by powers of two) where the chain's layer-0 input is register-resident or pre-transformed,
 * else split bf16 (6 MFMAs per product); others (and tuning mlp_f32 = 1) use the fp32 MFMA
 * kernels. */
int64_t pn2_layer_split_kblocks(int64_t cin, int64_t xyz);
int64_t pn2_layer_split_bytes(int64_t cout, int64_t cin, int64_t xyz);
int pn2_pack_layer_split_bf16(const float *W, int64_t cout, int64_t cin, int64_t xyz,
                              int xyz_first, void *out, void *stream);

/* Side job of an SA MLP call (pn2_sa_src.fps_side): the NEXT SA layer's farthest point sampling
 * -- pn2_fps_host_ws_f32's arguments, start_host[B] in host memory (read during the call).  It
 * runs inside the call's chain launch as extra workgroups when that launch allows it (its layer-0
 * input register-resident; B <= 256 clouds of N <= 512 points with C = 3 or 10, S <= 8192, its
 * LDS within the chain's), overlapping the MLP, else as its own launch on the same stream; the
 * same results either way.  Its inputs must not be written by the call; it needs no workspace
 * (pn2_fps_workspace_bytes == 0, else PN2_EINVAL).  In the reference the next layer samples
 * after this one's MLP (pointnet2_cls_ssg.py:27-28; the same draw order, the draws taken on the
 * host before the call). */
typedef struct pn2_fps_side {
    const float *pts; int64_t B, N, C, sb, sn, sc; /* points[b,n,c] = pts[b*sb + n*sn + c*sc]  */
    const int64_t *start_host;                      /* [B], host memory                       */
    int64_t S;
    int64_t *out_idx; float *out_pts; float *out_packed; float *pts_packed; /* as pn2_fps_f32 */
} pn2_fps_side;

typedef struct pn2_sa_src {
    int mode; /* PN2_SRC_* */
    const float *pts; int64_t pb, pn, pc; /* points [B,N,C], any strides            */
    const float *feat; int64_t fb, fn;    /* features [B,N,D], channel stride 1, or NULL */
    const float *ctr;                     /* centroids [B,S,C] contiguous (group modes) */
    const int64_t *idx;                   /* [B,S,K] int64 contiguous (group modes)     */
    const float *rows; int64_t rs;        /* PN2_SRC_ROWS: [M][rs]                      */
    int64_t B, N, C, D, S, K;             /* rows M = B*S*K (GROUP_ALL: S=1, K=N)       */
    const int32_t *cnt;                   /* [B,S] distinct neighbours per group
                                             (pn2_ball_query_cnt_f32), or NULL: group
                                             modes then compute only those rows          */
    float *zero_out; int64_t zero_count;  /* side job, or NULL: zero_count floats to zero
                                             (group_all's new_points, the reference's
                                             torch.zeros(B,1,C), pointnet2_utils.py:136),
                                             done by one of the call's launches          */
    const int32_t *idx32;                 /* [B,S,K] int32 (pn2_ball_query_i32), read in
                                             place of idx when not NULL (group modes)    */
    const pn2_fps_side *fps_side;         /* side job, or NULL (see pn2_fps_side)        */
} pn2_sa_src;

/* Bytes of workspace pn2_sa_mlp_max_f32 needs for this layer chain: 0 when the chain runs as
 * one fused kernel (every hidden width <= 256 and a compiled tile signature), otherwise two
 * [M][max hidden width] float32 buffers for the layer-by-layer path.  -1 on invalid input. */
int64_t pn2_sa_mlp_workspace_bytes(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                   int nlayers);

/* Fused gather -> nlayers x (1x1 conv + BN + ReLU) -> output.
 *   pool != 0 : out[g*ostride + c] = max over the K rows of group g (g = b*S+s) -- the
 *               torch.max(new_feature, 2)[0] of the reference, stored channels-last.
 *   pool == 0 : out[row*ostride + c] (dense rows, feeds a following PN2_SRC_ROWS call).
 * nlayers in [1,4]; every cout must be a multiple of 32.  Hidden activations stay in LDS; the
 * last layer is computed in 256-column slices (and split over the grid when nlayers == 1).
 * workspace may be NULL when pn2_sa_mlp_workspace_bytes() returns 0. */
int pn2_sa_mlp_max_f32(const pn2_sa_src *src, const pn2_mlp_layer *layers, int nlayers,
                       int pool, float *out, int64_t ostride, float *workspace,
                       int64_t workspace_bytes, void *stream);

/* The same fused SA MLP in bf16 arithmetic (BASELINE config 5, "features/MLP in bf16"):
 * every layer reads its input rounded to bf16 (round-to-nearest-even) and the hi plane of its
 * pn2_pack_layer_split_bf16 image (= bf16(W)); products are exact, accumulation, BN, ReLU and
 * the max are fp32, `out` is fp32.  Same arguments as pn2_sa_mlp_max_f32; every layer needs
 * wt_split.  Chains the register-resident chain kernel or the dense-layer kernel do not cover
 * return PN2_EUNSUPPORTED (no silent fp32 fallback).  Workspace: the _bf16 size query.
 * Replaces nothing in the reference (it has no bf16 path): same interface as
 * model/pointnet2_utils.py:167-172 at a lower precision, chosen by the caller. */
int64_t pn2_sa_mlp_workspace_bytes_bf16(const pn2_sa_src *src, const pn2_mlp_layer *layers,
                                        int nlayers);
int pn2_sa_mlp_max_bf16(const pn2_sa_src *src, const pn2_mlp_layer *layers, int nlayers,
                        int pool, float *out, int64_t ostride, float *workspace,
                        int64_t workspace_bytes, void *stream);

/* ---- input preparation (the step before the path) ----
 * pts: a DataLoader batch as float64 [B,N,C] (np.loadtxt rows), element (b,n,c) at
 * pts[b*sb + n*sn + c*sc].  For every cloud b, in float64 with numpy's operation order:
 *   mean_out[b*C + c] (or NULL) = float32(np.mean(points[b, :3, c]))  -- the first 3 POINTS, as
 *       test_translation.py:73 takes them, before normalising
 *   normalize != 0: xyz' = (xyz - centroid) / max_n |xyz_n - centroid|  (provider.normalization:
 *       centroid = sequential row sum / N, |v| = sqrt((x*x + y*y) + z*z)); C >= 3
 *   out[(b*N + n)*(C+K) + c] = float32(xyz'_c) (c < 3), float32(p[c]) (3 <= c < C),
 *       1.0f if c - C == labels[b] else 0.0f (C <= c < C+K, K = num_category; 0 = no splice)
 * out is the [B,N,C+K] float32 storage whose transpose(2,1) view is the model input (the
 * layout the reference's scripts hand the model).  labels: int64 [B] device, each in [0, K)
 * (checked by the caller: the reference raises IndexError).  1 <= C <= 64. */
int pn2_prepare_points_f64(const double *pts, int64_t B, int64_t N, int64_t C, int64_t sb,
                           int64_t sn, int64_t sc, int normalize, const int64_t *labels,
                           int64_t num_category, float *out, float *mean_out, void *stream);

/* ---- training (batch-statistics BatchNorm) around library GEMMs; rows are channels-last
 * [M][C] with row stride ld.  Workspace: pn2_bn_train_workspace_bytes(M, C) bytes (float64
 * chunk partials), caller-owned. ----
 * Column statistics of Y: mean, invstd = 1/sqrt(var_biased + eps); sxhat[c] = sum_r xhat
 * (float64, for the conv bias gradient); when momentum > 0 also
 * running_mean/var = (1-momentum)*old + momentum*(mean, var_unbiased) (torch's rule). */
int64_t pn2_bn_train_workspace_bytes(int64_t M, int64_t C);
int pn2_bn_train_stats_f32(const float *Y, int64_t M, int64_t C, int64_t ld, double eps,
                           double momentum, float *running_mean, float *running_var, float *mean,
                           float *invstd, double *sxhat, void *ws, int64_t ws_bytes, void *stream);
/* A = relu((Y - mean) * invstd * gamma + beta); flags PN2_LAYER_NO_RELU: no ReLU. */
int pn2_bn_relu_apply_f32(const float *Y, int64_t M, int64_t C, int64_t ld, const float *mean,
                          const float *invstd, const float *gamma, const float *beta, float *A,
                          int64_t lda, int flags, void *stream);
/* pn2_bn_train_stats_f32 then pn2_bn_relu_apply_f32 in one call (one host crossing per layer):
 * stats = [mean | invstd], 2*C floats. */
int pn2_bn_train_forward_f32(const float *Y, int64_t M, int64_t C, int64_t ld, double eps,
                             double momentum, float *running_mean, float *running_var,
                             const float *gamma, const float *beta, float *A, int64_t lda, int flags,
                             float *stats, double *sxhat, void *ws, int64_t ws_bytes, void *stream);
/* out[g*ldo + c] = max over k < K of A[(g*K + k)*lda + c]; arg[g*C + c] = first argmax (int32);
 * NaN is the maximum (first NaN), as torch.max. */
int pn2_group_max_f32(const float *A, int64_t G, int64_t K, int64_t C, int64_t lda, float *out,
                      int64_t ldo, int32_t *arg, void *stream);
/* Backward of A = relu(bn_train(Y)): dXn = dA * [A > 0] (dA with flags PN2_LAYER_NO_RELU, the
 * backward of A = bn_train(Y)), with dA dense (ldd) or, when dA is
 * NULL, scattered from the max: dA[r][c] = dOut[r/K][c] if arg[r/K][c] == r%K else 0.
 * dbeta = sum_r dXn, dgamma = sum_r dXn*xhat (float64 sums), and
 * dY = gamma*invstd*(dXn - dbeta/M - xhat*dgamma/M); dbias (or NULL) = sum_r dY, the preceding
 * conv's bias gradient, from the forward's sxhat. */
int pn2_bn_relu_backward_f32(const float *Y, int64_t M, int64_t C, int64_t ld, const float *mean,
                             const float *invstd, const float *gamma, const float *beta,
                             const float *dA, int64_t ldd, const float *dOut, int64_t ldo,
                             const int32_t *arg, int64_t K, const double *sxhat, float *dY,
                             int64_t ldy, float *dgamma, float *dbeta, float *dbias, void *ws,
                             int64_t ws_bytes, int flags, void *stream);

/* ---- small-batch fully connected layer (the eval FC tails, BN folded into W / bias on the
 * host): out[b*ldo + n] = act(sum_k x[b*ldx + k] * W[n*K + k] + bias[n]) for b < B (rows in
 * blocks of 16; each element computed the same way whatever B is),
 * W row-major [N][K], bias may be NULL; flags PN2_LINEAR_RELU applies the ReLU.  Float32 FMA.
 * Reference: pointnet_utils.py:33-40, pointnet_cls.py:26-28, rotation.py:45-49. ---- */
#define PN2_LINEAR_RELU 1
int pn2_linear_rows_f32(const float *x, int64_t ldx, int64_t B, int64_t K, const float *W,
                        const float *bias, float *out, int64_t ldo, int64_t N, int flags,
                        void *stream);

/* ---- the PointNet++ heads' eval FC tail in three launches: fc1 + bn1 + ReLU, fc2 + bn2 + ReLU
 * (as pn2_linear_rows_f32), then fc3 fused with the classifiers' log_softmax over the N3 logits
 * and the first argmax of each row (PN2_TAIL_LOGSOFTMAX) -- pointnet2_cls_ssg.py:31-38
 * (F.log_softmax(x, -1), x.data.max(1)[1]), the same tails of pointnet2_cls_msg.py,
 * rotation_ssg.py, translation_ssg.py, sign_ssg.py.  BN is folded into W / bias on the host;
 * dropout is the identity in eval.  x [B][K] (row stride ldx), W1 [N1][K], W2 [N2][N1],
 * W3 [N3][N2] row-major; out [B][N3] (row stride ldo): the log-probabilities with the flag, else
 * the fc3 outputs; argmax [B] int64 or NULL.  fc1 and fc2 elements are computed as
 * pn2_linear_rows_f32 computes them; each fc3 element is the in-order sum of four float32 fma
 * chains over consecutive quarters of k (the same whatever B is).  N3 <= 819.  workspace:
 * pn2_fc_tail_workspace_bytes(B, N1, N2) bytes, 16-byte aligned (y1 and y2). */
#define PN2_TAIL_LOGSOFTMAX 1
int64_t pn2_fc_tail_workspace_bytes(int64_t B, int64_t N1, int64_t N2);
int pn2_fc_tail_f32(const float *x, int64_t ldx, int64_t B, int64_t K, const float *W1,
                    const float *b1, int64_t N1, const float *W2, const float *b2, int64_t N2,
                    const float *W3, const float *b3, int64_t N3, int flags, float *out,
                    int64_t ldo, int64_t *argmax, void *workspace, int64_t workspace_bytes,
                    void *stream);

/* Which kernel family served this thread's last successful pn2_sa_mlp_max_* call:
 * PN2_PATH_F32 (fp32 MFMA kernels), PN2_PATH_SPLIT_BF16 (split-bf16 chain / dense kernels) or
 * PN2_PATH_BF16 (pn2_sa_mlp_max_bf16). */
#define PN2_PATH_F32 1
#define PN2_PATH_SPLIT_BF16 2
#define PN2_PATH_BF16 3
int pn2_sa_mlp_last_path(void);
/* Planes per operand of the MLP kernels of this thread's last successful pn2_sa_mlp_max_* call:
 * 3 (split bf16: 6 MFMAs per product), 2 (split fp16: 3), 1 (bf16), 0 (fp32 MFMA kernels). */
int pn2_sa_mlp_last_planes(void);
/* Where this thread's last pn2_sa_mlp_max_* call ran its FPS side job (pn2_sa_src.fps_side):
 * 1 inside the chain launch (extra workgroups of that launch), 0 as its own launch after the
 * MLP, -1 the call had no side job (ABI 17). */
int pn2_sa_mlp_last_fps_side(void);

/* ---- runtime: CU-partitioned streams (pipelined serving, pn2/pipeline.py) ---- */
int pn2_device_cu_count(int device, int *count);
/* A stream whose kernels run only on the CUs set in mask (bit i of word i/32 = CU i). */
int pn2_stream_create_cu_masked(int device, const uint32_t *mask, int mask_words, void **stream);
int pn2_stream_destroy(void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PN2_H */
