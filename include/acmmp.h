/*
 * acmmp.h — C-ABI of the MI355X-native ACMMP PatchMatch engine (libacmmp_amd.so).
 *
 * This is the drop-in boundary for the reference's hot path, `ACMMP::RunPatchMatch`
 * (src/ACMMP.cu:1378-1456) and the class surface around it (src/ACMMP.h:58-124).
 * Every entry point below names the reference member / function it replaces.
 * Plain C: POD structs, raw pointers + sizes, status-code returns, no exceptions,
 * no exit(): the reference's CUDA_SAFE_CALL -> exit(EXIT_FAILURE)
 * (src/ACMMP.cpp:67-75) becomes a negative status + acmmp_last_error().
 *
 * Image / map layout (host side): row-major float32, one array per view, size
 * height*width (the reference's cv::Mat_<float>). Plane hypotheses: row-major
 * float4 (x, y, z, w) = 4 floats per pixel, exactly the reference's
 * `float4 *plane_hypotheses_host` (src/ACMMP.h:97).
 */
#ifndef ACMMP_H_
#define ACMMP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACMMP_MAX_IMAGES 33   /* ref + up to 32 sources: the reference's unsigned
                                 selected_views bitmask and [32] arrays
                                 (src/ACMMP.cu:437, :805) */

/* Status codes */
#define ACMMP_OK 0
#define ACMMP_ERR_ARG -1
#define ACMMP_ERR_STATE -2
#define ACMMP_ERR_HIP -3
#define ACMMP_ERR_IO -4
#define ACMMP_ERR_UNSUPPORTED -5

/* == struct Camera (src/acmmp_definitions.h:47-55): K, R, t row-major, t is
 * world->camera, 100 bytes. */
typedef struct acmmp_camera {
    float K[9];
    float R[9];
    float t[3];
    int32_t height;
    int32_t width;
    float depth_min;
    float depth_max;
} acmmp_camera;

/* == struct PatchMatchParams (src/ACMMP.h:32-56) + the pinned RNG key.
 * Booleans are int32 for ABI stability. Defaults: acmmp_default_params(). */
typedef struct acmmp_params {
    int32_t max_iterations;     /* 2 in this fork (src/ACMMP.h:33) */
    int32_t patch_size;         /* 11 */
    int32_t num_images;         /* set by the image setters */
    int32_t max_image_size;     /* 3200 */
    int32_t radius_increment;   /* 2 */
    float sigma_spatial;        /* 5 */
    float sigma_color;          /* 3 */
    int32_t top_k;              /* 4 */
    float baseline;             /* 0.54 */
    float depth_min;
    float depth_max;
    float disparity_min;
    float disparity_max;
    float scaled_cols;
    float scaled_rows;
    int32_t geom_consistency;
    int32_t planar_prior;
    int32_t multi_geometry;
    int32_t hierarchy;
    int32_t upsample;
    int32_t seeded;
    uint32_t seed_lo;           /* Philox key: replaces curand_init(clock64(), ...) */
    uint32_t seed_hi;           /*   (src/ACMMP.cu:624), see include/acmmp_detmath.h */
    uint32_t rng_stream;        /* run index: a second RunPatchMatch on the same
                                   instance re-seeds like the reference's clock64() */
    int32_t texture_filter8;    /* 0 (default): pin A4, fp32 bilinear fractions. 1: the
                                   CUDA texture unit's 1.8 fixed-point fractions
                                   (cudaFilterModeLinear, src/ACMMP.cpp:659, used at
                                   src/ACMMP.cu:394): frac rounded to 1/256 before the
                                   lerp — an emulation (the hardware's sum order is not
                                   documented), for fidelity studies; oracle and GPU agree
                                   bit-exactly in both modes */
    int32_t reserved[4];
} acmmp_params;

/* Per-kernel timing of the last run, measured with hipEvents recorded on the
 * engine's own stream (enabled by acmmp_set_timing). Milliseconds. */
typedef struct acmmp_timing {
    float init_ms;          /* RandomInitialization */
    float sweep_ms;         /* sum over all Black/Red CheckerboardPropagation launches */
    int32_t sweep_launches; /* 2 * max_iterations */
    float finalize_ms;      /* GetDepthandNormal + Black/Red filter */
    float total_ms;         /* whole RunPatchMatch, device side */
} acmmp_timing;

/* == struct Problem (src/acmmp_definitions.h:57-63), fixed-size source list. */
typedef struct acmmp_problem {
    int32_t ref_image_id;
    int32_t num_src_images;
    int32_t src_image_ids[ACMMP_MAX_IMAGES - 1];
    int32_t max_image_size;     /* 6400 until ComputeMultiScaleSettings */
    int32_t num_downscale;
    int32_t cur_image_size;     /* 6400 until the scale loop sets it */
} acmmp_problem;

/* The flags of ProcessProblem (src/acmmp_definitions.cpp:245-250) plus what the
 * reference takes from globals: device (cudaSetDevice(0), :253), the RNG key
 * (clock64() in the reference) and an iteration override. */
typedef struct acmmp_pass_options {
    int32_t device;
    int32_t geom_consistency;
    int32_t planar_prior;
    int32_t hierarchy;
    int32_t multi_geometry;
    int32_t seeded;             /* pSampler seeded plane priors (src/acmmp_definitions.cpp:8-177, :275-281):
                                 * acmmp_prior_plane_estimate + SetPlanarPrior before the first RunPatchMatch */
    int32_t max_iterations;     /* <= 0: reference behaviour (2; SetGeomConsistencyParams forces 2) */
    uint32_t seed_lo;           /* Philox key of this pass */
    uint32_t seed_hi;
    int32_t write_triangulation;/* write 2333_%08d/triangulation.png in planar passes (:310-330) */
    int32_t verbose;            /* print the reference's progress lines to stdout */
    int32_t reserved[5];
} acmmp_pass_options;

typedef struct acmmp_ctx acmmp_ctx;

/* Fills the reference defaults of PatchMatchParams (src/ACMMP.h:32-56). */
void acmmp_default_params(acmmp_params *p);

/* ~ `ACMMP acmmp;` (src/acmmp_definitions.cpp:260) + cudaSetDevice(0) (:253):
 * create an engine bound to HIP device `device` with its own stream. */
int acmmp_create(int device, acmmp_ctx **out);
/* ~ ACMMP::~ACMMP (src/ACMMP.cpp:109-152). NULL is a no-op. Synchronises the
 * engine's own stream only (not the device, as the reference's cudaFree calls
 * do): work the caller queued on OTHER streams that still reads this engine's
 * buffers (acmmp_get_device_results pointers, band halo buffers) must be
 * finished before this call. After a clean sync the engine's device blocks,
 * stream and events go to a per-process cache for the next engine on the
 * device (at most ACMMP_DEVICE_POOL_MB MiB of blocks, default 8192; 0 or a
 * negative value turns the cache off); after a failed sync they are freed. */
void acmmp_destroy(acmmp_ctx *ctx);
/* Gives the device-block cache of `device` (every device: -1) back to the
 * HIP runtime with hipFree, plus the cached streams, events and host staging
 * blocks (the reference frees everything in its destructor; this returns the
 * memory the cache kept beside, e.g., torch's caching allocator). Blocks of
 * live engines are not touched. A hipMalloc that fails for lack of memory
 * releases the device's cache and retries once by itself. */
int acmmp_release_device_cache(int device);
/* Bytes of device blocks the cache currently holds for `device` (-1: all). */
int64_t acmmp_device_cache_bytes(int device);
/* Last error message on this context ("" when none). Never NULL. */
const char *acmmp_last_error(const acmmp_ctx *ctx);

int acmmp_set_params(acmmp_ctx *ctx, const acmmp_params *p);
int acmmp_get_params(const acmmp_ctx *ctx, acmmp_params *p);

/* ~ ACMMP::SetGeomConsistencyParams(bool) (src/ACMMP.cpp:447-454): sets
 * geom_consistency, forces max_iterations = 2, sets multi_geometry if asked. */
int acmmp_set_geom_consistency_params(acmmp_ctx *ctx, int multi_geometry);
/* ~ ACMMP::SetPlanarPriorParams (src/ACMMP.cpp:461-464). */
int acmmp_set_planar_prior_params(acmmp_ctx *ctx);
/* ~ ACMMP::SetHierarchyParams (src/ACMMP.cpp:456-459). */
int acmmp_set_hierarchy_params(acmmp_ctx *ctx);

/* In-memory equivalent of InputInitialization + CudaSpaceInitialization
 * (src/ACMMP.cpp:525-636, :638-681): upload `num_images` grayscale float
 * images (index 0 = reference view) and their (already rescaled) cameras.
 * Sets params.num_images and, like InputInitialization (:600-601), derives
 * depth_min = cams[0].depth_min*0.6, depth_max = cams[0].depth_max*1.2 unless
 * `keep_depth_range` is non-zero. images[i] has cams[i].height*cams[i].width
 * floats. Allocates all per-pixel device state for the reference size. */
int acmmp_set_images(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams,
                     const float *const *images, int keep_depth_range);

/* Geometric-consistency inputs (src/ACMMP.cpp:608-635, :683-743): the depth
 * map of every view (index 0 = ref, i = source i), each sized like that view,
 * host pointers. */
int acmmp_set_depth_maps(acmmp_ctx *ctx, const float *const *depths);
/* Same, BORROWING device buffers already resident on this engine's device
 * (e.g. slices of an RCCL all-gather): no copy; the caller keeps them alive and
 * unchanged until the run completes. pitches in floats (NULL = width). */
int acmmp_set_depth_maps_device(acmmp_ctx *ctx, const float *const *d_depths,
                                const int32_t *pitches);

/* Zero-copy variant of acmmp_set_images: the engine BORROWS the caller's
 * device-resident images (row pitch in floats, NULL = width). Inputs stay in
 * HBM across views and passes; nothing crosses PCIe. */
int acmmp_set_images_device(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams,
                            const float *const *d_images, const int32_t *pitches,
                            int keep_depth_range);

/* ~ cudaCreateTextureObject of one view (src/ACMMP.cpp:640-662): the padded
 * bilinear-footprint records of a device-resident grayscale image (row pitch
 * in floats), in the most compact form it fits, built once on `device` and
 * borrowed by every engine and run that uses the image, so no run re-pads it.
 * The image stays the caller's and must outlive the texture's use. */
typedef struct acmmp_texture acmmp_texture;
int acmmp_texture_create(int device, const float *d_image, int pitch, int width, int height,
                         acmmp_texture **out);
/* ~ cudaDestroyTextureObject (src/ACMMP.cpp:122-128). NULL is a no-op. */
void acmmp_texture_destroy(acmmp_texture *tex);
/* Bits per texel of the records: 8 (u8 quads), 16 (f16) or 32 (fp32). */
int acmmp_texture_bits(const acmmp_texture *tex);
/* acmmp_set_images_device from textures (index 0 = reference view): the
 * engine borrows their images and records. Textures of different forms are
 * re-padded per engine in their common form, as acmmp_set_images_device does. */
int acmmp_set_images_textures(acmmp_ctx *ctx, int num_images, const acmmp_camera *cams,
                              const acmmp_texture *const *textures, int keep_depth_range);

/* Previous-pass state for the reuse init branch (src/ACMMP.cpp:718-742):
 * planes = (world-frame normal xyz, depth) float4 per ref pixel, costs per pixel. */
int acmmp_set_plane_hypotheses(acmmp_ctx *ctx, const float *planes4, const float *costs);
/* Same from device buffers (copied device-to-device on the engine stream).
 * The engine stream does NOT wait for other streams: work that produced the
 * buffers on another stream must be complete, or ordered first with
 * acmmp_wait_stream. */
int acmmp_set_plane_hypotheses_device(acmmp_ctx *ctx, const float *d_planes4, const float *d_costs);

/* Orders the engine stream after everything enqueued so far on `stream` (a
 * hipStream_t of the same device; NULL = the legacy default stream): an event
 * recorded on `stream` that the engine stream waits on, no host wait. Every
 * *_device setter borrows or copies caller buffers on the engine stream,
 * which is created non-blocking; a producer on another stream (a torch
 * collective, a torch copy) must be ordered with this call first. The
 * reference has one blocking default stream and needs no such call
 * (src/ACMMP.cpp:638-831). */
int acmmp_wait_stream(acmmp_ctx *ctx, void *stream);

/* Hierarchy inputs (src/ACMMP.cpp:745-808): low-res scaled planes
 * (normal xyz + cost-or-depth in w) of size scaled_h*scaled_w, and the
 * upsampled depth for every ref pixel (plane_hypotheses[center].w, :797-804).
 * Sets params.upsample using the reference's test (:766), including its
 * rows/cols swap. */
int acmmp_set_hierarchy_inputs(acmmp_ctx *ctx, const float *scaled_planes4, int scaled_w,
                               int scaled_h, const float *upsampled_depth);
/* Same from device buffers (the view-parallel driver keeps them resident):
 * copied / expanded on the engine stream, ordered before the next run. */
int acmmp_set_hierarchy_inputs_device(acmmp_ctx *ctx, const float *d_scaled_planes4, int scaled_w,
                                      int scaled_h, const float *d_upsampled_depth);

/* ~ ACMMP::SetPlanarPrior(unique_ptr<float4>) (src/ACMMP.cpp:476-523): seeded
 * plane priors, float4 per ref pixel (camera-frame normal, distance). Sets
 * params.seeded. */
int acmmp_set_seed_prior(acmmp_ctx *ctx, const float *planes4);

/* ~ ACMMP::CudaPlanarPriorInitialization(vector<float4>, Mat_<float> mask)
 * (src/ACMMP.cpp:811-831): triangle planes (float4 each) and the per-pixel
 * triangle label mask (0 = none, k = plane k-1). */
int acmmp_set_planar_prior(acmmp_ctx *ctx, const float *plane_params4, int num_planes,
                           const uint32_t *mask);

/* ~ ACMMP::GetSupportPoints (src/ACMMP.cpp:868-894) on the resident results
 * of the last run: per 5x5 block (col-major block order) the pixel of lowest
 * cost < 2, kept if that cost < 0.1. Writes (x, y) pairs; *count = number
 * found (ACMMP_ERR_ARG if it exceeds capacity). */
int acmmp_get_support_points(acmmp_ctx *ctx, int32_t *xy, int capacity, int *count);

/* ~ ACMMP::DelaunayTriangulation (src/ACMMP.cpp:896-918): host-side exact
 * Delaunay triangulation of integer points inside [0,width) x [0,height)
 * (cv::Subdiv2D's bounding triangle, strict in-circle ties). Writes the
 * triangles with all three corners in the image, 6 int32 each
 * (x1 y1 x2 y2 x3 y3); needs no context or GPU. */
int acmmp_delaunay_triangulation(int width, int height, const int32_t *xy, int num_points, int32_t *tris,
                                 int capacity, int *num_triangles);

/* The planar-prior block of ProcessProblem (src/acmmp_definitions.cpp:332-376):
 * triangle raster into a label mask, ACMMP::GetPriorPlaneParams per triangle
 * (src/ACMMP.cpp:920-953) fitted to the resident depth map,
 * GetDepthFromPlaneParam range check (:955-958) and
 * CudaPlanarPriorInitialization (:811-831), all on the device. Optional
 * outputs: the fitted planes (float4 per kept triangle) and the final label
 * mask (W*H). Does not set params.planar_prior. */
int acmmp_build_planar_prior(acmmp_ctx *ctx, const int32_t *tris, int num_triangles, float *out_planes4,
                             uint32_t *out_mask);

/* Support points -> Delaunay -> acmmp_build_planar_prior ->
 * SetPlanarPriorParams (src/ACMMP.cpp:456-459), i.e. everything ProcessProblem
 * does between its two RunPatchMatch calls except the triangulation.png
 * drawing. */
int acmmp_prepare_planar_prior(acmmp_ctx *ctx, int *num_support_points, int *num_triangles);

/* ~ RunJBU + JBU_cu (src/ACMMP.cpp:1008-1087, src/ACMMP.cu:1458-1549): joint
 * bilateral upsampling of a low-res depth map (depth_width x depth_height)
 * to the reference image's size (width x height, the image already resized
 * to the current scale), on `device`. *image_scale receives
 * max(height / depth_height, width / depth_width); when it is 1 nothing is
 * computed or written, as in the reference. Host buffers in and out. */
int acmmp_joint_bilateral_upsample(int device, const float *image, int width, int height, const float *depth,
                                   int depth_width, int depth_height, float *out, int *image_scale);
/* Same on device buffers (row-major, unpadded): d_image width x height,
 * d_depth depth_width x depth_height, d_out width x height. Returns when
 * d_out is written. */
int acmmp_joint_bilateral_upsample_device(int device, const float *d_image, int width, int height,
                                          const float *d_depth, int depth_width, int depth_height, float *d_out,
                                          int *image_scale);

/* ~ ACMMP::RunPatchMatch (src/ACMMP.cu:1378-1456): init, max_iterations x
 * (black, red) checkerboard sweeps, depth/normal conversion, black/red median
 * filter. Results stay resident on the device; then rng_stream += 1. */
int acmmp_run_patchmatch(acmmp_ctx *ctx);
/* Asynchronous variant: enqueues the same work on the engine's stream and
 * returns without synchronising (for multi-view pipelining / benchmarks). */
int acmmp_run_patchmatch_async(acmmp_ctx *ctx);
/* Waits for all work enqueued on the engine's stream. */
int acmmp_synchronize(acmmp_ctx *ctx);

/* ---- Row-band split of ONE RunPatchMatch over several engines / ranks
 * (SURVEY §5 "image-size scaling": the reference has no intra-image split).
 * Each participant runs acmmp_run_patchmatch_band on the same inputs with
 * its own rows [row_lo, row_hi) of the reference image (the bands tile
 * 0..H). The sweeps compute only those rows; a pixel's CheckerboardPropagation
 * reads neighbour state up to ACMMP_BAND_HALO rows away (the far searches,
 * src/ACMMP.cu:819-826: 3 + 2 * 10 rows), so after every half-sweep the
 * engine calls `exchange` with the colour just written: the participant
 * must send its rows [send_*_lo, send_*_hi) of that colour's state to the
 * band above / below and receive theirs into rows [recv_*_lo, recv_*_hi)
 * (empty ranges where there is no neighbour). State rows are colour-split
 * (Wh elements per pixel row: plane float4, cost float, selected-views
 * u32). Initialisation runs on the band plus the halo rows (every pixel's
 * start is a function of its own inputs: the halos start valid), depth /
 * normal conversion and the two median filters on the band plus the rows the
 * filters read. Results (acmmp_get_* / acmmp_export_results) are valid for
 * rows [row_lo, row_hi) and bit-identical to acmmp_run_patchmatch's there.
 * Synchronous: returns when the run is complete. */
#define ACMMP_BAND_HALO 23
typedef struct acmmp_band_halo {
    int32_t colour;       /* checkerboard colour just written (0 black, 1 red) */
    int32_t Wh;           /* state elements per pixel row */
    void *plane;          /* float4 [H][Wh]: the colour's current planes (device) */
    void *cost;           /* float  [H][Wh] */
    void *sv;             /* u32    [H][Wh] */
    void *stream;         /* the engine's hipStream_t: enqueue on it, or synchronise it first */
    int32_t send_up_lo, send_up_hi;      /* own rows the band above reads */
    int32_t send_down_lo, send_down_hi;  /* own rows the band below reads */
    int32_t recv_up_lo, recv_up_hi;      /* rows of the band above this band reads */
    int32_t recv_down_lo, recv_down_hi;  /* rows of the band below this band reads */
} acmmp_band_halo;
typedef int (*acmmp_band_exchange_fn)(void *user, const acmmp_band_halo *halo);
int acmmp_run_patchmatch_band(acmmp_ctx *ctx, int row_lo, int row_hi, acmmp_band_exchange_fn exchange, void *user);

/* Bulk getters replacing the per-pixel GetPlaneHypothesis(int)/GetCost(int)
 * loops (src/ACMMP.cpp:848-856, src/acmmp_definitions.cpp:287-295).
 * `n` = capacity in elements (float4 count / float count / u32 count). */
int acmmp_get_plane_hypotheses(acmmp_ctx *ctx, float *planes4, size_t n);
int acmmp_get_costs(acmmp_ctx *ctx, float *costs, size_t n);
int acmmp_get_selected_views(acmmp_ctx *ctx, uint32_t *views, size_t n);
/* Device-resident result pointers (valid until the next set_images/destroy):
 * row-major float4 planes (world normal, depth) and float costs. */
int acmmp_get_device_results(acmmp_ctx *ctx, const float **d_planes4, const float **d_costs);

/* Device-to-device export of the last run's results into caller buffers
 * (any may be NULL): planes4 (W*H float4), costs (W*H), depth (W*H, the .w
 * channel — what depths.dmb holds). Enqueued on the engine stream; call
 * acmmp_synchronize before another stream reads them. */
int acmmp_export_results(acmmp_ctx *ctx, float *d_planes4, float *d_costs, float *d_depth);

/* ~ GetReferenceImageWidth/Height (src/ACMMP.cpp:833-841), GetCamera (:960-962),
 * GetMinDepth/GetMaxDepth (:858-866). */
int acmmp_get_reference_size(const acmmp_ctx *ctx, int *width, int *height);
int acmmp_get_camera(const acmmp_ctx *ctx, int index, acmmp_camera *cam);

/* Kernel-level evaluation used by the T1 parity tier: for every ref pixel and
 * the given camera-frame plane hypothesis (float4 per pixel), compute the cost
 * of every source view (ComputeMultiViewCostVector, src/ACMMP.cu:473-478)
 * -> out[(y*W+x)*(N-1) + v]; and if out_init is non-NULL the initial cost and
 * selected-view mask (ComputeMultiViewInitialCostandSelectedViews,
 * src/ACMMP.cu:434-471). */
int acmmp_eval_costs(acmmp_ctx *ctx, const float *planes4, float *out_costs,
                     float *out_init_cost, uint32_t *out_init_views);
/* ComputeGeomConsistencyCost (src/ACMMP.cu:518-543) for every pixel and view
 * -> out[(y*W+x)*(N-1) + v]. Needs depth maps. */
int acmmp_eval_geom_costs(acmmp_ctx *ctx, const float *planes4, float *out);

/* hipEvent timing of the next runs (on the engine stream). */
int acmmp_set_timing(acmmp_ctx *ctx, int enable);
int acmmp_get_timing(const acmmp_ctx *ctx, acmmp_timing *t);

/* Hardware self-test: compares v_rcp_f32 + one Newton step with the IEEE
 * division 1/z for every float32 in the fast-reciprocal exponent window
 * (2^-125 <= |z| < 2^125). mismatches == 0 proves the sweep's fast reciprocal
 * bit-identical to the pinned division on this device. */
int acmmp_selftest_reciprocal(int device, uint64_t *mismatches, uint64_t *checked);

/* Texel storage the gather kernels use for the current images (set by
 * acmmp_set_images*): 8 = u8 quads (the default whenever every view is
 * integer-valued in [0, 255], e.g. 8-bit JPEG input), 16 = f16 difference
 * quads (every stored value exact in f16, or ACMMP_TEXEL=h16), 32 = fp32 row
 * pairs (any other input, or ACMMP_TEXEL=f32). Results are identical in
 * every form; this reports the memory format only. No reference counterpart
 * (diagnostic). */
int acmmp_get_texel_bits(const acmmp_ctx *ctx);

/* Number of visible HIP devices (0 when none / no driver). */
int acmmp_device_count(void);
/* Library build string (arch, flags). */
const char *acmmp_version(void);
/* Host threads the library's thread pools use (image decodes, fusion, the
 * view-parallel driver's loads): the smallest of the affinity mask, the
 * cgroup CPU quota and OMP_NUM_THREADS (the launcher's declared budget);
 * ACMMP_HOST_THREADS overrides. The reference is single-threaded apart from
 * the OpenMP PLY writer (src/ACMMP.cpp:405). */
int acmmp_host_threads(void);

/* ---- Pass driver: the reference's pipeline around RunPatchMatch
 *      (src/acmmp_definitions.cpp:179-403, src/ACMMP.cpp:525-809), reading
 *      <dense>/images/%08d.jpg, <dense>/cams/%08d_cam.txt, <dense>/pair.txt and
 *      writing <out>/2333_%08d/{depths[_geom],normals,costs}.dmb. Host code in
 *      the library; the compute runs through the engine above. ---- */

/* ~ GenerateSampleList (src/acmmp_definitions.cpp:179-205): parse pair.txt,
 * dropping sources with score <= 0. *count = number of problems. */
int acmmp_generate_sample_list(const char *dense_folder, acmmp_problem *problems, int capacity, int *count);
/* ~ ComputeMultiScaleSettings (src/acmmp_definitions.cpp:207-243): per problem
 * max_image_size (capped at 3200) and num_downscale (halvings until <= 1000);
 * *max_num_downscale = the largest. */
int acmmp_compute_multiscale_settings(const char *dense_folder, acmmp_problem *problems, int count,
                                      int *max_num_downscale);
/* ~ ACMMP::InputInitialization (src/ACMMP.cpp:525-636): read the ref and source
 * images and cameras of problems[idx], rescale each to its problem's
 * cur_image_size (sources use problems[src_id], as the reference does), set
 * the depth range, and in geometric passes load the depth maps of the
 * previous pass. Parameters (geom / multi_geometry / hierarchy) must be set
 * before. */
int acmmp_input_initialization(acmmp_ctx *ctx, const char *dense_folder, const char *output_folder,
                               const acmmp_problem *problems, int count, int idx);
/* One view of InputInitialization (src/ACMMP.cpp:536-598): reads
 * images/%08d.jpg and cams/%08d_cam.txt of `image_id`, sets the camera's size
 * and rescales image + K to max_image_size when larger. *cam is always
 * filled on success of the read; `out` receives cam->width*cam->height floats
 * when capacity suffices (else ACMMP_ERR_ARG). */
int acmmp_load_view(const char *dense_folder, int image_id, int max_image_size, float *out, size_t capacity,
                    acmmp_camera *cam);
/* ~ ACMMP::CudaSpaceInitialization (src/ACMMP.cpp:638-809): previous-pass
 * plane/cost state of the reference view (geometric passes) and the
 * hierarchy inputs (low-res normals/costs + upsampled depth). */
int acmmp_space_initialization(acmmp_ctx *ctx, const char *output_folder, const acmmp_problem *problem);
/* ~ ProcessProblem (src/acmmp_definitions.cpp:245-403): one view of one pass,
 * including the planar-prior second run, written as .dmb files. */
int acmmp_process_problem(const char *dense_folder, const char *output_folder, const acmmp_problem *problems,
                          int count, int idx, const acmmp_pass_options *options);
/* ~ JointBilateralUpsampling (src/acmmp_definitions.cpp:405-438): upsample
 * 2333_%08d/depths_geom.dmb to the image resized to acmmp_size, overwriting
 * 2333_%08d/depths.dmb. */
int acmmp_joint_bilateral_upsampling(const char *dense_folder, const char *output_folder,
                                     const acmmp_problem *problem, int acmmp_size, int device);
/* ~ pSampler::pSampler / confirm_using_prior (src/acmmp_definitions.cpp:8-29,
 * 91-93): 1 when <dense>priors/{depths,normals}/%08d.png of camera
 * num_cams-1 can be read (the path is dense_folder + "priors", as in the
 * reference), else 0. */
int acmmp_priors_available(const char *dense_folder, int num_cams);
/* ~ pSampler::GetPriorPlaneEstimate (src/acmmp_definitions.cpp:99-177): the
 * seeded plane prior of camera `cam_num` at rows x cols from the 16-bit depth
 * (mapped to [cam.depth_min, depth_max]) and normal (mapped to [-1, 1], BGR)
 * PNGs, through depth_normal_to_plane (:72-89) — including normVec3's
 * multiplication by the norm. float4 per pixel, row-major. */
int acmmp_prior_plane_estimate(const char *dense_folder, int cam_num, const acmmp_camera *cam, int rows, int cols,
                               float *planes4);

/* ~ RunFusion (src/acmmp_definitions.cpp:828-1043): fuse the depth_geom (or
 * depth) + normal maps of all problems into <output>/ACMMP_model.ply (binary
 * PLY of StoreColorPlyFileBinaryPointCloud, src/ACMMP.cpp:382-424), colours
 * from <dense><image_dir>/%08d.jpg; optional masks <dense>/<mask_folder>/
 * %08d.png (" " = none, as the reference); write_debug_images writes
 * <dense>/approved_pixels_cam_%d.png. Sequential and literal (the
 * reference's order dependence included). Host code. */
int acmmp_run_fusion(const char *dense_folder, const char *output_folder, const acmmp_problem *problems, int count,
                     int geom_consistency, float consistency_scalar, int con_num_thresh, const char *image_dir,
                     const char *mask_folder, int write_debug_images, int *num_points);
/* ~ RunPriorAwareFusion (src/acmmp_definitions.cpp:573-826): fuses the maps
 * of `fusion_folder` with this run's (`output_folder`) seeded maps as priors,
 * per pixel choosing the hypothesis with more consistent views
 * (single_match_penalty for one-sided support), into
 * <output>/ACMMP_prior_model.ply. Host code, literal. The reference's
 * mask_folder argument (:579, :657-666) is not taken: its mask is
 * `Mat_<Vec3b>(imread(path, -1)) < 128`, i.e. 0 / 255, and the walk skips a
 * pixel only where the mask byte == 1, which only its own approvals write, so
 * a readable mask file changes nothing (an unreadable one crashes it). */
int acmmp_run_prior_aware_fusion(const char *dense_folder, const char *output_folder, const char *fusion_folder,
                                 const acmmp_problem *problems, int count, int geom_consistency,
                                 float consistency_scalar, int num_consistent_thresh, int single_match_penalty,
                                 int *num_points);
/* Message of the last failing acmmp_run_fusion / _prior_aware_fusion on this thread. */
const char *acmmp_fusion_last_error(void);

/* Message of the last failing driver call on this thread ("" when none). */
const char *acmmp_pipeline_last_error(void);

/* ~ ACMMP::GetReferenceImage (src/ACMMP.cpp:843-846): the (rescaled) reference
 * image, width*height floats. */
int acmmp_get_reference_image(acmmp_ctx *ctx, float *out, size_t n);
/* ~ ACMMP::GetPriorPlaneParams (src/ACMMP.cpp:920-953) for one triangle
 * (x1 y1 x2 y2 x3 y3) with the depths at its corners; host. */
int acmmp_prior_plane_params(const acmmp_camera *cam, const int32_t *tri, const float *depths, float *out4);
/* ~ ACMMP::GetDepthFromPlaneParam (src/ACMMP.cpp:955-958); host. */
float acmmp_depth_from_plane_param(const acmmp_camera *cam, const float *plane4, int x, int y);

/* ---- Reference on-disk formats (src/ACMMP.cpp:154-380,
 *      src/acmmp_definitions.cpp:179-205). Pure host code. ---- */

/* ~ cv::imread(path, cv::IMREAD_GRAYSCALE) + convertTo(CV_32FC1) as used by
 * InputInitialization (src/ACMMP.cpp:538-541, :553-556): baseline JPEG
 * (luminance plane, libjpeg ISLOW IDCT), binary PGM (P5) or grayscale PFM.
 * Writes width*height floats (row-major) when capacity suffices; otherwise
 * returns ACMMP_ERR_ARG with *width / *height set. */
int acmmp_read_image_gray(const char *path, float *out, size_t capacity, int *width, int *height);
/* ~ cv::imread(path, cv::IMREAD_COLOR) as RunFusion uses it
 * (src/acmmp_definitions.cpp:858): baseline JPEG decoded like libjpeg
 * (fancy chroma upsampling, fixed-point YCbCr->RGB) or an 8-bit PNG;
 * width*height*3 bytes in BGR order when capacity suffices, else
 * ACMMP_ERR_ARG with the size set. */
int acmmp_read_image_bgr(const char *path, uint8_t *out, size_t capacity, int *width, int *height);
/* Image dimensions from the file header only (ComputeMultiScaleSettings,
 * src/acmmp_definitions.cpp:219-224, decodes the whole image for this). */
int acmmp_image_size(const char *path, int *width, int *height);
/* ~ cv::imread(path, IMREAD_UNCHANGED) of a non-interlaced 8/16-bit gray,
 * gray+alpha, RGB or RGBA PNG: samples widened to uint16, colour channels in
 * OpenCV's BGR(A) order. Writes width*height*channels values when capacity
 * suffices; otherwise ACMMP_ERR_ARG with the dimensions set. */
int acmmp_read_png(const char *path, uint16_t *out, size_t capacity, int *width, int *height, int *channels,
                   int *bit_depth);
/* ~ cv::resize(src, dst, Size(dst_width, dst_height), 0, 0, INTER_LINEAR) on
 * a float image (src/ACMMP.cpp:589): half-pixel centres, edge clamp,
 * horizontal pass first; an exact 2x downscale is the 2x2 mean (OpenCV's
 * INTER_AREA fast path). */
int acmmp_resize_linear(const float *src, int src_width, int src_height, float *dst, int dst_width,
                        int dst_height);

/* ReadCamera (src/ACMMP.cpp:154-179). width/height are left 0. */
int acmmp_read_camera(const char *path, acmmp_camera *cam);
/* readDepthDmb / readNormalDmb (src/ACMMP.cpp:264-294, :323-353): on success
 * fills h, w, nb; if data != NULL copies min(cap, h*w*nb) floats. */
int acmmp_read_dmb(const char *path, int32_t *h, int32_t *w, int32_t *nb, float *data,
                   size_t cap);
/* writeDepthDmb / writeNormalDmb (src/ACMMP.cpp:296-321, :355-380). */
int acmmp_write_dmb(const char *path, int32_t h, int32_t w, int32_t nb, const float *data);

#ifdef __cplusplus
}
#endif

#endif /* ACMMP_H_ */
