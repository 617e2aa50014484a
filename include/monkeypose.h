/* monkeypose.h -- C ABI of libmonkeypose.so, the MI355X (gfx950) inference path of the
 * monkey-pose regressors.
 *
 * The reference (krg-nandu/monkey-pose, TensorFlow 1.x / Python 2) has no FFI: its "operator API"
 * is a set of Python graph-builder classes.  Each entry point below replaces one of them; the
 * Python facade in monkey-pose_amd/ (hgru_pose.py, hgru_module.py) binds them with ctypes and
 * keeps the reference's class / method names and argument order.
 *
 *   reference interface                                        replaced by
 *   ---------------------------------------------------------  ------------------------------------
 *   hgru_pose.model.get_var / data_dict   hgru_pose.py:196-216  mp_set_weight, mp_finalize_weights
 *   hgru_pose.model.build(depth, output_shape, batch_norm,     mp_hgru_pose_fwd
 *     train_mode) -> .out_put             hgru_pose.py:47-105
 *   hgru_module.ContextualCircuit(X, timesteps, SRF, SSN, SSF, mp_hgru_circuit_fwd
 *     strides, padding, aux).build()      hgru_module.py:61-128, 872-959
 *   (tf.Session / device placement)       train_cnn_networks_hgru.py:95  mp_create / mp_destroy
 *
 * Conventions
 *   - Every tensor argument is a device pointer (hipMalloc'd or a torch CUDA tensor's data_ptr),
 *     fp32, contiguous, NHWC exactly as the reference feeds it (depth crops [n,128,128,1] =
 *     crop_mm / 10000, train_cnn_networks_hgru.py:50).  Output buffers are caller-owned.
 *   - Weights are identified by their TensorFlow variable names (e.g. "cnn/contextual_circuit/p_r",
 *     "cnn/fc_1/fc_1_weights"); a leading "cnn/" scope is optional.  The library copies them.
 *   - Calls on one context are serialised by the caller and are asynchronous on `stream`
 *     (a hipStream_t; NULL = default stream).  One context per device.
 *   - Status: MP_OK (0) or a negative MP_ERR_*; mp_last_error() gives a thread-local message.
 *     No C++ exception crosses the ABI.  Shapes are validated on the host before any launch.
 */
#ifndef MONKEYPOSE_H
#define MONKEYPOSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mp_ctx mp_ctx;

enum {
  MP_OK = 0,
  MP_ERR_ARG = -1,         /* bad argument / null pointer */
  MP_ERR_STATE = -2,       /* weights missing or not finalized */
  MP_ERR_HIP = -3,         /* HIP runtime error (message has hipGetErrorString) */
  MP_ERR_WEIGHT = -4,      /* unknown weight name or wrong shape */
  MP_ERR_SHAPE = -5,       /* unsupported input shape */
  MP_ERR_UNSUPPORTED = -6  /* option not implemented (e.g. train_mode) */
};

enum {
  MP_MODEL_HGRU_POSE = 1,    /* hgru_pose.model                (hgru_pose.py:6-216)        */
  MP_MODEL_HGRU_CIRCUIT = 2, /* hgru_module.ContextualCircuit  (hgru_module.py:54-959)     */
  MP_MODEL_DENSE = 3,        /* dense_model_struct  (train_dense_networks.py:211-509)      */
  MP_MODEL_HIER = 4,         /* hier_model_struct   (train_hier_networks.py:327-631)       */
  MP_MODEL_ATTN = 5,         /* attn_model_struct   (train_cnn_networks_hgru.py:422-525)   */
  MP_MODEL_GRAPH = 6         /* a recorded layer graph (mp_graph_set): dense_hier_model_struct
                                (train_dense_hier_networks.py:327-2507)                       */
};

enum { MP_MEM_HOST = 0, MP_MEM_DEVICE = 1 };
/* compute precision of the hGRU association-field convolutions (the rest of the path is fp32):
 *   MP_DTYPE_F32        exact fp32 (v_mfma_f32_32x32x2_f32, an fmaf chain)
 *   MP_DTYPE_F32_SPLIT  fp32-accurate "f16x3": each fp32 operand split into two power-of-two
 *                       scaled f16 halves (22 mantissa bits), three f16 MFMAs per product with fp32
 *                       accumulation; errors within a few fp32 ulps of the F32 path, 5.3x fewer
 *                       matrix-core cycles.  Needs map height and width multiples of 32.
 *   MP_DTYPE_F32_FFT    fp32 FFT convolution on a 72x72 grid (exact circular = SAME linear conv
 *                       for maps up to 64x64): fp32 72-point FFTs + a per-frequency complex
 *                       channel GEMM in the f16x3 split (three v_mfma_f32_32x32x16_f16 per complex
 *                       MAC term, fp32 accumulation); ~50x fewer FLOPs than direct at 15x15 taps,
 *                       error ~1e-6 of max|output|.  Needs map height <= 64, width 32 or 64.
 *   MP_DTYPE_BF16       the FFT path with bf16 spectra (input and output), bf16 spectral weights and
 *                       bf16 1x1 gate weights: one v_mfma_f32_32x32x16_bf16 product per MAC, fp32
 *                       accumulation, fp32 FFTs and elementwise math; the hGRU maps O / I / Og / P2
 *                       and the drive X stored as bf16; conv_2 / conv_3 and fc_1 run one f16
 *                       product per MAC (hi x hi of the f16x3 split, fp32 accumulation); conv_1,
 *                       the BNs and the fc_1 output stay fp32.  Error ~1e-3 of max|output| on the
 *                       pose (gate 5e-3), a few 1e-3 on the raw circuit state (SURVEY config 4). */
enum { MP_DTYPE_F32 = 0, MP_DTYPE_F32_SPLIT = 1, MP_DTYPE_F32_FFT = 2, MP_DTYPE_BF16 = 3 };

/* library version, (major << 16) | minor */
int mp_version(void);

/* thread-local description of the last error on this thread ("" if none) */
const char* mp_last_error(void);

/* create a context on HIP device `device` for model `model_kind` */
int mp_create(int device, int model_kind, mp_ctx** out);
void mp_destroy(mp_ctx* ctx);

/* copy one variable (fp32, row-major, TF shape) into the context; replaces
 * hgru_pose.get_var / tf.get_variable (hgru_pose.py:196-216, hgru_module.py:262-503) */
int mp_set_weight(mp_ctx* ctx, const char* name, const float* data, const int64_t* shape, int ndim,
                  int mem_kind);

/* replicate the weights set on ctxs[root] (mp_set_weight) into every other context of the list --
 * one per device, or several on one device -- device to device, as a binomial tree of peer copies
 * over xGMI: ceil(log2(nctx)) rounds, each round doubling the contexts that hold the weights, every
 * copy of a round in flight together, nothing staged through the host.  Each context then runs
 * its own mp_finalize_weights.  For one process driving several GPUs (SURVEY 8b's proposed
 * weight broadcast); one process per GPU broadcasts the blob with torch.distributed (RCCL) instead
 * (monkey-pose_amd/parallel.py).  Replaces loading data_dict / get_var once per device
 * (hgru_pose.py:196-216). */
int mp_bcast_weights(mp_ctx* const* ctxs, int nctx, int root);

/* fold BN, pack every weight into its kernel's fragment order; must follow the last
 * mp_set_weight and precede any forward call */
int mp_finalize_weights(mp_ctx* ctx, int compute_dtype);

/* pre-allocate the activation workspace for batches up to max_batch (otherwise grown lazily) */
int mp_reserve(mp_ctx* ctx, int64_t max_batch);

/* ContextualCircuit aux 'hidden_init' (hgru_module.py:875-892): the initial output state O0.
 * The initial I is never read by the hgru_pose aux (795-804). */
enum {
  MP_HIDDEN_GIVEN = 0,    /* o0 as passed ('random' with the caller's draw, e.g. for parity)  */
  MP_HIDDEN_ZEROS = 1,    /* O0 = zeros_like(X)                      (888-890); o0 unused */
  MP_HIDDEN_IDENTITY = 2, /* O0 = X, the circuit's drive             (876-878); o0 unused */
  MP_HIDDEN_RANDOM = 3    /* 'random' (879-887): a fresh draw on the device per call, xavier-uniform
                             with limit sqrt(6 / (k + k)); element i of the NHWC O0 is
                             f32((2u - 1) * limit), u = splitmix64(i * 0x9E3779B97F4A7C15 + key) >> 11
                             scaled by 2^-53, key = fnv1a64("h2_init") ^ (s * 0x2545F4914F6CDD1D),
                             s = rng_seed + rng_call (monkey-pose_amd/weights.py synth_hidden(seed=s)) */
};

/* hgru_pose.model.build (hgru_pose.py:47-105), inference:
 *   depth  [n, h, w, 1]   normalised depth crops (h = w = 128 in the reference)
 *   o0     [n, h/2, w/2, 64] initial hGRU output state (hidden_init='random',
 *          hgru_module.py:879-887, made explicit)
 *   out    [n, output_shape] joint coordinates / (cube_z / 2), joint-major (j*3 + {x,y,z}) */
int mp_hgru_pose_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w,
                     const float* o0, float* out, void* stream);

/* the reference model's readable intermediates (hgru_pose.py:50-103: m.conv1, m.pool1, m.conv2,
 * m.conv3, m.hgru, m.fc1, m.relu1); each a caller-owned device buffer, NULL = not wanted.
 * NHWC fp32 like the reference tensors; [n, 1024] for fc1 / relu1.  (The 0.1 layout; 0.2 keeps it.) */
typedef struct {
  float* conv1;  /* [n, h, w, 64]      relu(conv_1)                       (50)      */
  float* pool1;  /* [n, h/2, w/2, 64]  BN(max_pool(conv1))                (51-60)   */
  float* conv2;  /* [n, h/2, w/2, 64]  BN(relu(conv_2))                   (61-70)   */
  float* conv3;  /* [n, h/2, w/2, 64]  BN(relu(conv_3))                   (71-80)   */
  float* hgru;   /* [n, h/2, w/2, 64]  BN(O_T), the fc_1 input            (81-90)   */
  float* fc1;    /* [n, 1024]          fc_1 + bias (pre-activation)       (91)      */
  float* relu1;  /* [n, 1024]          BN(relu(fc1))                      (92-103)  */
} mp_pose_taps;

/* per-call options of mp_hgru_pose_fwd_ex / mp_hgru_circuit_fwd_opts (since 0.2).  struct_size =
 * sizeof(mp_fwd_opts) as the caller was compiled: the library reads that many bytes and no more,
 * and fields added by later versions keep their defaults for older callers.  Zero-initialise. */
typedef struct {
  uint64_t struct_size;
  int32_t hidden_init;        /* MP_HIDDEN_*; o0 may be NULL unless MP_HIDDEN_GIVEN */
  int32_t reserved;
  uint64_t rng_seed;          /* MP_HIDDEN_RANDOM: the draw of seed rng_seed + rng_call */
  uint64_t rng_call;          /*   (the caller's per-call counter: the reference re-draws per run) */
  /* store_states (hgru_module.py:889-915): every timestep's states, [n, T, h/2, w/2, 64] NHWC
   * (the reference's stack transposed to batch-major, 909-912).  states_O[:, t] = O_t after the
   * rho gain, states_I[:, t] = I_t.  (The reference's own stacks swap O and I on alternate steps:
   * full() takes (store_O, store_I) where the loop passes (store_I, store_O), hgru_module.py:825,
   * 897-908; here each stack holds what its name says.)  NULL = not wanted. */
  float* states_O;
  float* states_I;
  const mp_pose_taps* taps;   /* pose model only: the intermediates, or NULL */
} mp_fwd_opts;

/* mp_hgru_pose_fwd with options (opts may be NULL: the mp_hgru_pose_fwd defaults) */
int mp_hgru_pose_fwd_ex(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, const float* o0,
                        float* out, const mp_fwd_opts* opts, void* stream);

/* mp_hgru_pose_fwd that also writes the requested intermediates (taps may be NULL) */
int mp_hgru_pose_fwd_taps(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w,
                          const float* o0, float* out, const mp_pose_taps* taps, void* stream);

/* ContextualCircuit(X, timesteps, ...).build() -> O  (hgru_module.py:872-959), hgru_pose aux:
 *   x, o0, o_out  [n, h, w, k] NHWC; k must be 64, h % 16 == 0, w % 32 == 0;
 *   timesteps <= the length of the "contextual_circuit/rho" weight */
int mp_hgru_circuit_fwd(mp_ctx* ctx, const float* x, const float* o0, int64_t n, int64_t h,
                        int64_t w, int64_t k, int timesteps, float* o_out, void* stream);

/* mp_hgru_circuit_fwd with the aux 'hidden_init' (MP_HIDDEN_GIVEN / _ZEROS / _IDENTITY; o0 may be
 * NULL unless MP_HIDDEN_GIVEN) and 'store_states' (hgru_module.py:889-915): states_O / states_I,
 * each [n, timesteps, h, w, k] NHWC or NULL, receive every step's O_t (after the rho gain) and I_t */
int mp_hgru_circuit_fwd_ex(mp_ctx* ctx, const float* x, const float* o0, int64_t n, int64_t h, int64_t w,
                           int64_t k, int timesteps, int hidden_init, float* o_out, float* states_O,
                           float* states_I, void* stream);

/* mp_hgru_circuit_fwd with every option of mp_fwd_opts except taps (since 0.2) */
int mp_hgru_circuit_fwd_opts(mp_ctx* ctx, const float* x, const float* o0, int64_t n, int64_t h, int64_t w,
                             int64_t k, int timesteps, float* o_out, const mp_fwd_opts* opts, void* stream);

/* dense_model_struct.build(depth, output_shape) -> .output  (train_dense_networks.py:223-408):
 *   depth [n, h, w, 1] (h, w multiples of 32 in the reference's 128x128), out [n, output_shape] */
int mp_dense_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, float* out,
                 void* stream);

/* hier_model_struct.build(depth, output_shape, P_shape, R_shape, M_shape, I_shape, T_shape)
 * (train_hier_networks.py:338-530): outs[0] = .output [n, output_shape], outs[1..5] =
 * .p_output .r_output .m_output .i_output .t_output [n, *_shape] (sizes = the fc_3 widths) */
int mp_hier_fwd(mp_ctx* ctx, const float* depth, int64_t n, int64_t h, int64_t w, float* const* outs,
                void* stream);

/* attn_model_struct.build(depth, output_shape) -> .out_put  (train_cnn_networks_hgru.py:436-525),
 * the attention (centre-of-mass) regressor, inference (BN from moving statistics, no dropout):
 *   frames [n, h, w, 1] normalised full depth frames (image / image_max_depth,
 *          train_cnn_networks_hgru.py:116; 424 x 512 in the reference), resized to 128 x 128
 *   out    [n, output_shape] (u, v, d) / (image_orig_size[0], image_orig_size[1], image_max_depth) */
int mp_attn_fwd(mp_ctx* ctx, const float* frames, int64_t n, int64_t h, int64_t w, float* out, void* stream);

/* tf.image.resize_images(x, [ho, wo]) with the TF1 defaults (BILINEAR, align_corners=False,
 * legacy source coordinates in = out * in_size / out_size), bit-identical to TF's float32 kernel:
 *   x [n, h, w, c] -> out [n, ho, wo, c], device pointers */
int mp_resize_bilinear(const float* x, int64_t n, int64_t h, int64_t w, int64_t c, int64_t ho, int64_t wo,
                       float* out, void* stream);

/* ---- host-side 3D CoM crop (no GPU; the pre-step of every regressor) -------------------------
 * MonkeyDetector(fx, fy, ux, uy, cube, d1, d2) (monkeydetector.py:31-63, tf_monkeydetector.py),
 * constructed in the reference as (365.456, 365.456, 256, 212, [800,800,1200], 200, 10000)
 * (train_cnn_networks_hgru.py:77). */
typedef struct {
  double fx, fy, ux, uy; /* focal lengths, principal point (pixels) */
  double cube[3];        /* crop volume (x, y, z) in mm */
  double min_depth;      /* d1: near plane, mm */
  double max_depth;      /* d2: far plane, mm (also the canvas fill of the crop) */
} mp_camera;

/* depth frame element type: float32 mm (the hGRU caller: image * 10000, train_cnn_networks_hgru.py:47)
 * or uint16 mm (Kinect PNG, sample_pipeline.py:21); numpy semantics differ and are kept: the CoM
 * depth sum is float32-pairwise vs exact, the near-plane clamp rounds vs truncates */
enum { MP_DEPTH_F32 = 0, MP_DEPTH_U16 = 1 };

/* MonkeyDetector.calculateCoM (monkeydetector.py:66-83): com = (mean col, mean row, sum(d)/count)
 * over pixels with min_depth <= d <= max_depth of a float32 [h][w] frame in mm; (0,0,0) if none */
int mp_center_of_mass(const mp_camera* cam, const void* depth, int depth_dtype, int64_t h, int64_t w,
                      double com[3]);

/* MonkeyDetector.cropArea3D(dpt, com, dsize=(dsize, dsize)) (monkeydetector.py:261-334):
 *   com     (u, v, d) in pixels / mm, or NULL to use mp_center_of_mass
 *   out     [dsize][dsize] float32 crop in mm, canvas filled with max_depth
 *   M       3x3 row-major crop transform (off * scale * trans), com_out: the CoM used
 *   info    optional {xstart, xend, ystart, yend, sz_w, sz_h, off_x, off_y} (integers of the crop) */
int mp_crop3d(const mp_camera* cam, const void* depth, int depth_dtype, int64_t h, int64_t w, const double* com,
              int64_t dsize, float* out, double M[9], double com_out[3], int32_t info[8]);

/* mp_crop3d with cropArea3D's other options (since 0.2):
 *   flags  MP_CROP_DOCOM: docom=True, the second refinement (monkeydetector.py:287-300) -- the CoM of
 *          the first crop (+ xstart / ystart), falling back to the crop's centre depth and then to
 *          300 mm when that CoM is (0,0,0), and a second crop around it; com_out is the refined CoM */
enum { MP_CROP_DOCOM = 1 };
int mp_crop3d_ex(const mp_camera* cam, const void* depth, int depth_dtype, int64_t h, int64_t w, const double* com,
                 int flags, int64_t dsize, float* out, double M[9], double com_out[3], int32_t info[8]);

/* prepare_data_test (train_cnn_networks_hgru.py:61-74) for n frames [n][h][w]: patches
 * [n][dsize][dsize][1] = crop / max_depth (the model input), Ms [n][9], coms_out [n][3];
 * coms [n][3] or NULL; frames are processed by up to nthreads host threads */
int mp_crop3d_batch(const mp_camera* cam, const void* frames, int depth_dtype, int64_t n, int64_t h, int64_t w,
                    const double* coms, int64_t dsize, float* patches, double* Ms, double* coms_out,
                    int nthreads);

/* prepare_data_test on the device (train_cnn_networks_hgru.py:61-74) with tr_res = the attention
 * output, for a batch of n frames in one launch (asynchronous; every pointer is device memory
 * except cam and com_scale, which are read on the host at the call):
 *   frames    [n][h][w] float32 as fed to the attention net; the crop sees frames * frame_scale
 *             (image_np * image_max_depth, line 67: frame_scale = 10000)
 *   com_norm  [n][3] float32 attention output; com = com_norm * com_scale in float64
 *             (com_scale: host double[3] = {image_orig_size[0], image_orig_size[1], image_max_depth},
 *             line 69)
 *   patches   [n][dsize][dsize][1] = cropArea3D(frame, com) / cam.max_depth
 *   Ms [n][9], coms_out [n][3] float64; status [n] int32: 0 ok, else the frame's crop failed
 *             (1 CoM depth zero / not finite, 2 empty crop, 3 degenerate bounds, 4 empty resize;
 *             that patch is all ones) -- the host mp_crop3d raises MP_ERR_ARG in those cases.
 * Integers (bounds, sizes, offsets, nearest-neighbour indices) are bit-exact with mp_crop3d. */
int mp_crop3d_dev(const mp_camera* cam, const float* frames, int64_t n, int64_t h, int64_t w, float frame_scale,
                  const float* com_norm, const double* com_scale, int64_t dsize, float* patches, double* Ms,
                  double* coms_out, int32_t* status, void* stream);

/* mp_crop3d_dev with flags (since 0.2): MP_CROP_DOCOM runs cropArea3D's docom refinement per frame on
 * the device (one block per frame: calculateCoM of the first crop with numpy's float32 pairwise
 * sum order, the allclose / isclose fallbacks, the second crop); coms_out then holds the refined
 * CoMs.  Bit-exact with mp_crop3d_ex(..., MP_CROP_DOCOM, ...). */
int mp_crop3d_dev_ex(const mp_camera* cam, const float* frames, int64_t n, int64_t h, int64_t w, float frame_scale,
                     const float* com_norm, const double* com_scale, int flags, int64_t dsize, float* patches,
                     double* Ms, double* coms_out, int32_t* status, void* stream);

/* read a model property: "output_shape", "timesteps", "ssf", "finalized", "workspace_bytes",
 * "weight_bytes", "fft_loop" (hGRU contexts: 4 = the four-step FFT loop, 6 = the six-launch FFT
 * loop, 0 = a direct-convolution dtype, no FFT path); graph contexts also "graph_kernels" (kernel launches per forward),
 * "graph_streams" (streams the schedule uses), "graph_buffers" (activation buffers after concat placement), "graph_fused_pools" (2x2 max pools
 * computed inside their conv's kernel: MP_GRAPH_FUSE / MP_GRAPH_FUSE_POOL) -- as planned by the
 * last forward */
int mp_info(mp_ctx* ctx, const char* key, int64_t* value);

/* per-kernel device timing with HIP events recorded on the launch stream around every launch of
 * kernel class `name` ("conv15_a", "conv15_b", "fc1", "backbone"); enable, run, then read the
 * summed elapsed milliseconds and launch count (reading synchronises those events) */
int mp_profile_enable(mp_ctx* ctx, int enable);
int mp_profile_read(mp_ctx* ctx, const char* name, double* total_ms, int64_t* launches);

/* ---- layer-graph runtime (MP_MODEL_GRAPH) ---------------------------------------------------
 * The reference's regressors are TF1 graph builders: build() chains conv_layer / max_pool /
 * tf.concat / fc_layer calls.  A facade records the same calls as ops (tensor ids in SSA order:
 * id 0 = the [n, h, w, in_channels] input, every op defines `out`); the library then plans and runs
 * the graph natively:
 *   - tf.concat is free: a weighted union-find places every concatenated tensor as a channel
 *     range of one wide NHWC buffer per concat group, which its producers write in place;
 *   - relu / identity fold into their producer (conv_layer already applies relu; a relu after
 *     fc_layer becomes the FC epilogue);
 *   - kernels run as a dependency DAG over up to MP_GRAPH_STREAMS (env, default 8) HIP streams.
 * Replaces the graph-builder half of dense_hier_model_struct.build (train_dense_hier_networks.py:
 * 338-2382; helpers conv_layer 2431-2446, max_pool 2426-2429, avg_pool 2416-2419, max_pool_4
 * 2421-2424, fc_layer 2448-2455). */
enum {
  MP_OP_CONV = 1,     /* relu(conv2d(src, name/name_filters, stride, SAME) + name/name_biases) */
  MP_OP_MAXPOOL = 2,  /* ksize x ksize / ksize max pool, SAME (ksize 2 or 4)                     */
  MP_OP_AVGPOOL = 3,  /* 2x2 / 2 average pool, SAME (in-image count)                             */
  MP_OP_CONCAT = 4,   /* tf.concat(src[0..n_src), axis=-1)                                       */
  MP_OP_FC = 5,       /* reshape(src, [-1, K]) @ name/name_weights + name/name_biases             */
  MP_OP_RELU = 6,     /* tf.nn.relu                                                              */
  MP_OP_IDENTITY = 7  /* tf.identity                                                             */
};
#define MP_GRAPH_MAX_SRC 8
typedef struct {
  int32_t kind;                    /* MP_OP_* */
  int32_t out;                     /* tensor id defined by this op (> every id it reads) */
  int32_t n_src;
  int32_t src[MP_GRAPH_MAX_SRC];
  int32_t ksize, stride, cout;     /* conv: filter size, stride, out channels; pools: ksize */
  const char* name;                /* conv / fc: the layer's variable scope ("dense_1_conv_1_scale_1") */
} mp_graph_op;

/* install the graph of an MP_MODEL_GRAPH context (before mp_finalize_weights, which packs every
 * conv / fc layer it names); outputs: the tensor ids mp_graph_fwd writes, in order */
int mp_graph_set(mp_ctx* ctx, const mp_graph_op* ops, int n_ops, int in_channels, const int32_t* outputs,
                 int n_outputs);

/* run the graph on x [n, h, w, in_channels]; outs[i] = caller-owned device buffer holding output
 * tensor i densely ([n, cout] for an fc output, [n, H, W, C] otherwise) */
int mp_graph_fwd(mp_ctx* ctx, const float* x, int64_t n, int64_t h, int64_t w, float* const* outs, void* stream);

/* ---- HBM streaming probe (diagnostic; bench.py's practical roof) ----------------------------
 * The box's streaming HBM rates over `bytes`-sized buffers (>= 64 MiB; 2 GiB recommended):
 * read-only, write-only and copy (read + write bytes / time), each the best over grids of 1024 -
 * 8192 blocks of 256 threads, 1 / 4 / 8 16-byte accesses per thread in flight and default or
 * non-temporal policy (the chosen form is reported).  The ceiling the HBM-bound FFT-path kernels
 * are read against, next to the 8 TB/s spec figure.  Synchronous; not on any product path. */
typedef struct {
  double read_gbps, write_gbps, copy_gbps;
  int32_t read_grid, read_unroll, read_nt;
  int32_t write_grid, write_unroll, write_nt;
  int32_t copy_grid, copy_unroll, copy_nt;
} mp_hbm_rates;
int mp_hbm_probe(int device, int64_t bytes, mp_hbm_rates* out);

/* ---- TF1 checkpoint support (host only; monkey-pose_amd/tf_checkpoint.py) ----
 * CRC-32C (Castagnoli, reflected 0x82F63B78) of n bytes continuing from `init` (0 to start), as
 * tensor_bundle (BundleEntryProto.crc32c) and LevelDB-format table blocks store it before masking.
 * Replaces the checksum half of tf.train.NewCheckpointReader (train_cnn_networks_hgru.py:248-250,
 * 312-313: saver.restore). */
uint32_t mp_crc32c(uint32_t init, const void* data, size_t n);

/* ---- TFRecord ingestion (host only; monkey-pose_amd/data_loader.py) ----------
 * Replaces tf.TFRecordReader + tf.parse_single_example + tf.decode_raw (data_loader.py:10-26) and
 * tf.python_io.TFRecordWriter + encode_example (Datareader.py:13-27).  A reader memory-maps the
 * file and indexes its records once (length CRCs always checked, payload CRCs when verify != 0). */
typedef struct mp_tfrecord mp_tfrecord;
int mp_tfrecord_open(const char* path, int verify, mp_tfrecord** out, int64_t* n_records);
void mp_tfrecord_close(mp_tfrecord* r);
/* byte size of bytes feature `feature` (BytesList value[0], or a packed FloatList) of record rec */
int mp_tfrecord_feature_size(mp_tfrecord* r, int64_t rec, const char* feature, int64_t* bytes);
/* decode_raw gather: out[i] = the raw bytes of `feature` in record indices[i], each exactly
 * bytes_per_record (else MP_ERR_SHAPE), decoded by up to nthreads host threads */
int mp_tfrecord_read(mp_tfrecord* r, const int64_t* indices, int64_t count, const char* feature, void* out,
                     int64_t bytes_per_record, int nthreads);
/* write n_records tf.train.Example records {names[k]: bytes_feature(data[k] + i * bytes_per_record[k])}
 * (features in the given order), creating or (append != 0) extending the file */
int mp_tfrecord_write(const char* path, int64_t n_records, int n_features, const char* const* names,
                      const void* const* data, const int64_t* bytes_per_record, int append);

#ifdef __cplusplus
}
#endif

#endif /* MONKEYPOSE_H */
