/*
 * yolo_hip.h — C ABI of the MI355X (gfx950) YOLOv11 inference path.
 *
 * This is the drop-in boundary between the Python mirror of the reference's
 * module API (yolo-infer-pt_amd/nets/nn.py, yolo-infer-pt_amd/utils/util.py)
 * and the hand-written HIP kernels in yolo-infer-pt_amd/csrc/.  Signatures use
 * plain pointers and sizes only; no torch types cross this line.
 *
 * Reference interfaces replaced (file:line into t0saki/YOLO-Infer-pt):
 *   yh_create           nets/nn.py:308-347  yolo_v11_{n,t,s,m,l,x}() -> YOLO(width, depth, csp, nc)
 *                       nets/nn.py:282-292  YOLO.__init__ (DarkNet + DarkFPN + Head graph)
 *   yh_conv_count,
 *   yh_conv_info        the reference's state_dict naming (nets/nn.py module tree), one entry per conv
 *   yh_load_conv        nets/nn.py:8-25     fuse_conv (BN folded into conv in fp32), nets/nn.py:299-305 YOLO.fuse
 *   yh_forward          nets/nn.py:294-297  YOLO.forward in eval mode, incl. Head.forward decode
 *                       (nets/nn.py:255-270), DFL (nets/nn.py:222-225) and make_anchors (utils/util.py:85-96)
 *   yh_forward_u8       main.py:265-267     uint8 -> dtype, / 255 preprocessing fused into yh_forward's stem
 *   yh_nms              utils/util.py:123-169 non_max_suppression (+ torchvision.ops.nms, util.py:162)
 *   yh_nms_host         the same for head outputs on the CPU device (main.py:20 device fallback)
 *   yh_letterbox        utils/dataset.py:95-103, 292-313, 86-88: eval-mode load_image resize
 *                       (cv2 INTER_LINEAR) + zero border + HWC->CHW, BGR->RGB, on the device
 *   yh_letterbox_host   the same on the host (Dataset.__getitem__ in the loader workers)
 *
 * Conventions
 *   - Every function returns 0 on success and a negative YH_E* code on failure;
 *     yh_last_error() returns a thread-local message describing the last failure.
 *   - Device pointers are HIP device memory owned by the caller (PyTorch tensors).
 *     The library owns its packed weights and its activation workspace.
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream).
 *     yh_forward and yh_nms are asynchronous on that stream: they never
 *     synchronise the host and allocate nothing once the workspace for a
 *     given (batch, height, width) exists.
 *   - One handle is bound to one device and one compute dtype.  Calls on one
 *     handle must be serialised by the caller; distinct handles are independent
 *     (data-parallel serving = one handle per GPU).
 */
#ifndef YOLO_HIP_H
#define YOLO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YH_ABI_VERSION 5

/* status codes */
#define YH_OK 0
#define YH_EINVAL -1     /* bad argument / shape */
#define YH_ESTATE -2     /* call out of order (e.g. forward before all weights loaded) */
#define YH_EHIP -3       /* HIP runtime error */
#define YH_ENOMEM -4     /* device allocation failed */

/* compute / storage dtypes of a handle (activations and outputs) */
#define YH_F32 0
#define YH_F16 1
#define YH_BF16 2

typedef struct yh_handle yh_handle;

/* Network description: the (width, depth, csp) triple of nets/nn.py:308-347 plus
 * the class count (Head nc, nets/nn.py:232-238). */
typedef struct {
    int width[6];     /* e.g. {3,16,32,64,128,256} for v11_n */
    int depth[6];     /* repeat counts; only depth[0..5] as used by DarkNet/DarkFPN */
    int csp[2];       /* 0/1: C3k nesting for shallow / deep C3k2 blocks */
    int num_classes;  /* nc */
} yh_variant;

/* ABI version of the loaded library (YH_ABI_VERSION). */
int yh_abi_version(void);

/* Thread-local message of the last failing call ("" if none). */
const char* yh_last_error(void);

/* Build the layer graph of a variant for `device` in `dtype` (YH_F32/F16/BF16). */
int yh_create(const yh_variant* variant, int device, int dtype, yh_handle** out);

/* Release all device memory owned by the handle. NULL is accepted. */
void yh_destroy(yh_handle* h);

/* Number of convolutions whose weights the handle expects. */
int yh_conv_count(const yh_handle* h);

/* Describe conv `index`: `name` = state_dict prefix of the owning module
 * (e.g. "net.p2.1.res_m.0.conv1" for a Conv block, "head.box.0.2" for a plain
 * nn.Conv2d); shape of the expected fp32 weight (cout, cin_per_group, k, k);
 * `has_bias` = 1 if the reference module carries a conv bias (head output
 * convs). The pointer in *name stays valid for the handle's lifetime. */
int yh_conv_info(const yh_handle* h, int index, const char** name, int* cout,
                 int* cin_per_group, int* ksize, int* groups, int* has_bias);

/* Load one conv from host fp32 arrays. `weight` is (cout, cin/groups, k, k)
 * contiguous. `bias` may be NULL (treated as zeros). If `bn_gamma` is non-NULL
 * the BatchNorm (gamma, beta, running mean, running var, eps) is folded in
 * exactly as fuse_conv (nets/nn.py:8-25) does it, in fp32. Packed, dtype-cast
 * copies are uploaded to the handle's device; host arrays may be freed after. */
int yh_load_conv(yh_handle* h, int index, const float* weight, const float* bias,
                 const float* bn_gamma, const float* bn_beta, const float* bn_mean,
                 const float* bn_var, double bn_eps);

/* Anchors produced for an input of height x width (sum over strides 8/16/32). */
int yh_num_anchors(const yh_handle* h, int height, int width, int* anchors);

/* Bytes of device workspace the handle holds for (batch, height, width)
 * after yh_reserve (activations, excluding weights). */
int yh_workspace_bytes(const yh_handle* h, int batch, int height, int width, size_t* bytes);

/* Optional: allocate the workspace for (batch, height, width) up front. */
int yh_reserve(yh_handle* h, int batch, int height, int width);

/* Eval-mode forward.
 *   x: device (batch, 3, height, width) NCHW contiguous, handle dtype
 *   y: device (batch, 4 + nc, anchors) contiguous, handle dtype:
 *      rows 0..3 = (cx, cy, w, h) in pixels, rows 4.. = sigmoid class scores
 * height, width: multiples of 32. */
int yh_forward(yh_handle* h, const void* x, int batch, int height, int width,
               void* y, void* stream);

/* yh_forward on the data loader's image tensor: x is device (batch, 3, height,
 * width) NCHW uint8 (RGB, utils/dataset.py:86-88 layout), and the reference's
 * preprocessing `samples.half() / 255.` (main.py:265-267; to the handle dtype)
 * is fused into the stem's input load - no converted copy of x is made.
 * Bit-identical to yh_forward on x.to(dtype) / 255. computed by torch on the
 * device (u * fp32(1/255), rounded to the dtype). */
int yh_forward_u8(yh_handle* h, const void* x, int batch, int height, int width,
                  void* y, void* stream);

/* Bytes of device workspace yh_nms needs for a (batch, 4 + num_classes, anchors) input. */
size_t yh_nms_workspace_bytes(int batch, int num_classes, int anchors);

/* Batched NMS over a head output y (batch, 4 + num_classes, anchors) of dtype
 * YH_F32/F16/BF16, on the current HIP device. Stateless: the caller supplies the
 * workspace (yh_nms_workspace_bytes). Semantics of non_max_suppression
 * (utils/util.py:123-169): candidate (anchor, class) pairs with score >
 * conf_threshold (threshold rounded to the input dtype, as torch compares),
 * sorted by score descending (ties: lower anchor*nc + class first), truncated to
 * max_nms, class-offset boxes (class * max_wh), greedy IoU > iou_threshold
 * suppression (torchvision.ops.nms contract), at most max_det kept per image.
 *   dets:   device float (batch, max_det, 6) = x1, y1, x2, y2, score, class
 *   counts: device int32 (batch) kept detections per image
 * Box geometry is evaluated in fp32 for every dtype; class scores must lie in
 * [0, 2) (sigmoid outputs). Asynchronous on `stream`. */
int yh_nms(int dtype, const void* y, int batch, int num_classes, int anchors,
           float conf_threshold, double iou_threshold, int max_det, int max_nms,
           float max_wh, void* workspace, size_t workspace_bytes,
           float* dets, int* counts, void* stream);

/* The same NMS on the host CPU for a head output in HOST memory (the reference's
 * CPU device path, main.py:20): identical candidate / order / suppression rules,
 * torchvision's CPU loop in float32. dets (batch, max_det, 6) and counts (batch)
 * are host arrays; `threads` <= 0 uses every hardware thread (images in parallel).
 * Synchronous. */
int yh_nms_host(int dtype, const void* y, int batch, int num_classes, int anchors,
                float conf_threshold, double iou_threshold, int max_det, int max_nms,
                float max_wh, float* dets, int* counts, int threads);

/* Letterbox geometry of one image for a square canvas of `size` (dataset.py:95-103,
 * 292-313): resized height / width (int(h * r), int(w * r) with r = size / max(h, w);
 * unchanged when r == 1) and the top / left border. */
int yh_letterbox_geometry(int height, int width, int size, int* new_h, int* new_w, int* top, int* left);

/* Eval-mode preprocessing of a batch of decoded images, on the device:
 *   srcs[i]: device uint8 HWC BGR image of heights[i] x widths[i], row stride
 *            strides[i] bytes (strides may be NULL: 3 * width)
 *   dst:     device uint8 (batch, 3, size, size) RGB CHW: the image resized as
 *            cv2.resize INTER_LINEAR does (11-bit fixed point; exact 2x
 *            downscales as INTER_AREA) and centred on a zero border.
 * Asynchronous on `stream`. yh_letterbox_host computes the same bytes for one
 * image in host memory (dst (3, size, size)); `threads` > 1 splits the rows. */
int yh_letterbox(const void* const* srcs, const int* heights, const int* widths, const int* strides,
                 int batch, int size, void* dst, void* stream);
int yh_letterbox_host(const void* src, int height, int width, int stride, int size, void* dst, int threads);

/* cv2.resize(src, (new_w, new_h), INTER_LINEAR) of one uint8 HWC 3-channel host image
 * (the resize step alone; dst is new_h x new_w x 3, channel order kept). */
int yh_resize_linear_host(const void* src, int height, int width, int stride, int new_h, int new_w, void* dst);

/* Per-op instrumentation (bench / roofline). With profiling enabled,
 * yh_forward launches the ops eagerly with a HIP event pair around each op on
 * the caller's stream, synchronises at the end and accumulates per-op elapsed
 * milliseconds. Disabled by default (forward then runs as a HIP graph). */
int yh_profile_enable(yh_handle* h, int enable);
int yh_profile_reset(yh_handle* h);

/* Number of ops (kernel launch groups) in the forward. */
int yh_op_count(const yh_handle* h);

/* Describe op `index` for an input of (batch, height, width): label (module
 * path), class (0 dense 3x3 conv, 1 dense 1x1 conv, 2 stem conv, 3 depthwise,
 * 4 SPPF pools, 5 PSA attention, 6 head decode, 7 fused head cls branch,
 * 8 fused box tail with DFL, 9 fused C3k2 block, 10 fused C3k block, 11 fused box branch of all
 * levels), algorithmic bytes (each
 * operand read once, each output written once, handle dtype) and FLOPs per
 * call, accumulated profiled milliseconds and call count. */
int yh_op_info(const yh_handle* h, int index, int batch, int height, int width,
               const char** label, int* op_class, double* bytes, double* flops,
               double* ms_total, int* calls);

/* Use a captured HIP graph for yh_forward (default on). */
int yh_set_graph(yh_handle* h, int enable);

/* Kernel that runs op `index` at (batch, height, width): for a dense conv of a
 * 16-bit handle the conv_mx plan the per-shape tuner picked on the first
 * yh_forward at that shape (e.g. "mxr_k3s1_na2_mb2_b1x2_nb2"; every plan is
 * bit-identical), "gemm_f32" on the fp32 handle, for the other ops the op's
 * kernel name. YH_ESTATE before that forward. */
int yh_op_kernel(const yh_handle* h, int index, int batch, int height, int width, const char** name);

/* Force conv plan `kernel` (an index into each conv's candidate list, clamped)
 * on every dense conv, or -1 to return to per-shape autotuning. Drops the tuned
 * choices and captured graphs. Testing hook: every plan must produce
 * bit-identical outputs. */
int yh_force_conv_kernel(yh_handle* h, int kernel);

/* Launch units of the forward at (batch, height, width), known after the first
 * yh_forward at that shape: a unit is one op's kernel (is_level is always 0; the
 * fused level programs of ABI 1 are gone).
 * yh_unit_count returns the count (YH_ESTATE before that forward). With
 * yh_profile_enable, ms_total / calls accumulate per unit. */
int yh_unit_count(const yh_handle* h, int batch, int height, int width);
int yh_unit_info(const yh_handle* h, int index, int batch, int height, int width, int* first_op,
                 int* num_ops, int* is_level, double* ms_total, int* calls);

/* Parity taps (tests/test_gpu_op_parity.py; no reference counterpart: they expose the
 * per-module intermediates nets/nn.py:28-270 computes, so each fused / 16-bit kernel can be
 * checked against the fp64 oracle on its own device-produced inputs).
 *
 * yh_debug_op_desc writes a JSON description of op `index` at (batch, height, width) into buf
 * (NUL-terminated; returns its length, or a negative status): kind, label, "active" (1 if the
 * op launches at this shape, 0 if a fused alternative replaces it, -1 before the first
 * yh_forward there), the convs it computes ({name, k, s, g, act, cin, cout, bias}, in the
 * op's order, null for an absent one) and its workspace operands ({role, H, W, C, logical,
 * up}: inputs "in0"/"in1"/"res"/"x<l>"/"L<l>", outputs "out"/"y<l>"; an op whose output
 * is the caller's y, or whose input is the caller's x, lists no operand for it).
 *
 * yh_debug_run_ops launches the active ops in [first, last) eagerly on `stream`, after a
 * yh_forward at the same shape (x_u8: x is the uint8 image tensor). Running 0..n in steps
 * reproduces yh_forward's workspace and y exactly.
 *
 * yh_debug_operand copies operand `slot` (the desc's order) of op `index` out of the
 * workspace into dst as a dense (batch, H, W, C) array of the handle dtype, async on stream;
 * dst_bytes must equal that array's size at the workspace's current shape (YH_EINVAL otherwise). */
int yh_debug_op_desc(const yh_handle* h, int index, int batch, int height, int width, char* buf, size_t size);
int yh_debug_run_ops(yh_handle* h, const void* x, int x_u8, int batch, int height, int width, void* y, int first,
                     int last, void* stream);
int yh_debug_operand(const yh_handle* h, int index, int slot, void* dst, size_t dst_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* YOLO_HIP_H */
