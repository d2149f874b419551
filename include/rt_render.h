/*
 * rt_render.h — C-ABI drop-in boundary for the per-pixel render path of
 * tlinford/raytracer-challenge-rs (`Camera::render(&World) -> Canvas -> PPM`),
 * implemented by hand-written HIP kernels for MI355X (gfx950).
 *
 * Plain C types only: pointers, sizes, doubles. No torch, no HIP types in the
 * signatures (`stream` is an opaque hipStream_t passed as void*).
 *
 * Every entry point cites the reference interface it replaces
 * (paths relative to the reference repository root).
 *
 * Conventions
 *   - All matrices are 4x4, row-major, element (i,j) at [i*4+j]
 *     (reference `Matrix::idx`, raytracer/src/matrix.rs:75-77).
 *   - All arithmetic is IEEE-754 binary64 in the reference's operation order.
 *   - Return value: RT_OK (0) on success, a negative RT_ERR_* code otherwise;
 *     the message is available from rt_last_error() on the calling thread.
 *     The library never aborts across the ABI (the reference panics instead:
 *     raytracer/src/geometry/intersection.rs:113, matrix.rs:139, canvas.rs:45-46).
 *
 * Threads and devices (callable from any host thread)
 *   - Every entry point may be called from any host thread, on one scene or
 *     on several at once. An rt_scene's lock is held only while a call
 *     enqueues its work: the synchronous entry points (the host-buffer calls
 *     rt_render*, rt_render_ppm, rt_color_at_batch*, rt_is_shadowed_batch,
 *     rt_hit_batch, and any call given a non-NULL `stats`) wait for the device
 *     and copy their results without it, each in a context (stream, device
 *     buffers) of its own, so threads rendering one scene overlap on the GPU.
 *   - Asynchronous calls (rt_render_shard_device[_ex], rt_render_frames_device
 *     without stats) never wait on the host: every recursion generation of the
 *     frame sizes itself on the device, for a new camera as for a repeated one.
 *     Work issued on one stream runs in issue order; different streams overlap.
 *   - Every entry point that selects a scene's device restores the caller's
 *     current HIP device before it returns, on success and on failure.
 *   - rt_last_error() is per thread.
 */
#ifndef RT_RENDER_H
#define RT_RENDER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6

/* ---- status codes ------------------------------------------------------ */
enum {
  RT_OK = 0,
  RT_ERR_INVALID_ARGUMENT = -1,
  RT_ERR_UNSUPPORTED_SHAPE = -2,
  RT_ERR_HIP = -3,
  RT_ERR_RCCL = -4,
  RT_ERR_DUPLICATE_SHAPES = -5, /* structurally-equal shapes: see DESIGN.md */
  RT_ERR_NOT_INVERTIBLE = -6,   /* Matrix::inverse assert, matrix.rs:139 */
  RT_ERR_BUFFER_TOO_SMALL = -7,
  RT_ERR_NO_DEVICE = -8,
  RT_ERR_HOST = -9 /* host-side failure (e.g. out of host memory); no exception crosses the ABI */
};

/* ---- shape kinds / pattern kinds ---------------------------------------- */
enum {
  RT_SHAPE_SPHERE = 0,   /* geometry/shape/sphere.rs:16-77   */
  RT_SHAPE_PLANE = 1,    /* geometry/shape/plane.rs:19-64    */
  RT_SHAPE_CUBE = 2,     /* geometry/shape/cube.rs:17-106    */
  RT_SHAPE_CYLINDER = 3, /* geometry/shape/cylinder.rs:12-130 */
  RT_SHAPE_CONE = 4      /* geometry/shape/cone.rs:12-149    */
};

/* Anti-aliasing sample counts of `RenderOpts::aa_samples` (camera.rs:221-233). */
enum { RT_AA_X1 = 1, RT_AA_X2 = 2, RT_AA_X4 = 4, RT_AA_X8 = 8, RT_AA_X16 = 16 };
enum {
  RT_PATTERN_NONE = -1,
  RT_PATTERN_TEST = 0,     /* pattern/test_pattern.rs:7-9 */
  RT_PATTERN_STRIPE = 1,   /* pattern/stripe.rs:14-20     */
  RT_PATTERN_GRADIENT = 2, /* pattern/gradient.rs:14-18   */
  RT_PATTERN_RING = 3,     /* pattern/ring.rs:14-21       */
  RT_PATTERN_CHECKERS = 4  /* pattern/checkers.rs:14-21   */
};

/*
 * One flattened `Box<dyn Shape>` of `World::objects` (world.rs:18-21),
 * in the reference's object order. Fields mirror `BaseShape`
 * (geometry/mod.rs:12-20) and `Material` (material.rs:10-21).
 * `inverse` is `BaseShape::transform_inverse` as computed by the reference's
 * cofactor-expansion `Matrix::inverse` (matrix.rs:138-153); rt_matrix_inverse()
 * below computes exactly that. The transpose (`transform_inverse_transpose`)
 * is formed by the library.
 */
typedef struct rt_shape_desc {
  int32_t kind;            /* RT_SHAPE_* */
  int32_t casts_shadow;    /* BaseShape::shadow (geometry/mod.rs:19, :101-103) */
  double transform[16];    /* BaseShape::transform */
  double inverse[16];      /* BaseShape::transform_inverse */
  /* Material (material.rs:10-21) */
  double color[3];
  double ambient, diffuse, specular, shininess;
  double reflective, transparency, refractive_index;
  /* Material::pattern (Option<Pattern>, pattern/mod.rs:17-22) */
  int32_t pattern_kind;    /* RT_PATTERN_*, RT_PATTERN_NONE if None */
  int32_t _pad;
  double pattern_a[3], pattern_b[3];
  double pattern_transform[16];
  double pattern_inverse[16];
  /* Cylinder / Cone `minimum`, `maximum`, `closed` (cylinder.rs:12-18,
   * cone.rs:12-18); Cylinder::default / Cone::default = (-inf, +inf, false).
   * Ignored for the other kinds. */
  double minimum, maximum;
  int32_t closed;
  int32_t _pad2;
} rt_shape_desc;

/* (ABI 6) A `Group` (geometry/shape/group.rs:13-18) of the flattened World:
 * its bounding box as Group::intersect tests it (BaseShape::bounding_box of
 * the group, the union of its children's boxes, group.rs:71-94,128-133), and
 * the group that contains it (-1: a member of World::objects). Groups are
 * listed parents first. */
typedef struct rt_group_desc {
  double min[3], max[3];
  int32_t parent;
  int32_t _pad;
} rt_group_desc;

/* `PointLight` (light.rs:4-24), in `World::lights` insertion order. */
typedef struct rt_light_desc {
  double position[3];
  double intensity[3];
} rt_light_desc;

/* `Camera` (camera.rs:19-30) with its host-computed derived fields. */
typedef struct rt_camera_desc {
  uint32_t hsize, vsize;
  double pixel_size, half_width, half_height;
  double inverse[16]; /* Camera::transform_inverse */
} rt_camera_desc;

/* Work counters of one render call. One "ray" = one `World::intersect`
 * invocation of the reference (world.rs:71 for radiance rays, world.rs:101
 * for shadow rays); the `rays_*` and `*_tests` fields count the REFERENCE's
 * work and are exact on every path. The renders always run the fast path
 * (exact-culling BVH, shadow rays that cannot change a colour left out)
 * unless RT_RENDER_EXHAUSTIVE is passed to an `_ex` entry point; asking for
 * stats never changes the algorithm.
 *   sphere_tests / plane_tests / other_tests: the reference's loop tests
 *     every shape for every ray (world.rs:31-38), so these are rays x shapes.
 *   sphere_disc_ge0: sphere tests with disc >= 0 in the reference's loop.
 *     Only the exhaustive loop evaluates every one: RT_STATS_NOT_COUNTED on
 *     the fast path.
 *   *_traced / *_executed (ABI 3): what the kernels actually did. */
#define RT_STATS_NOT_COUNTED UINT64_MAX
typedef struct rt_stats {
  uint64_t rays_primary;
  uint64_t rays_reflect;
  uint64_t rays_refract;
  uint64_t rays_shadow;
  uint64_t sphere_tests;
  uint64_t plane_tests;
  uint64_t sphere_disc_ge0;
  uint64_t other_tests; /* Cube / Cylinder / Cone local_intersect calls */
  double ms_kernel; /* device time of the render kernel(s), HIP events */
  double ms_total;  /* wall time of the call */
  /* ABI 3 */
  uint64_t rays_shadow_traced;    /* shadow rays the kernels traced (<= rays_shadow) */
  uint64_t sphere_tests_executed; /* sphere tests the kernels executed (after culling) */
  uint64_t box_tests_executed;    /* BVH child-box tests executed */
  uint32_t exhaustive;            /* 1: rendered by the reference's every-shape loop */
  uint32_t _pad;
} rt_stats;

/* Flags of the `_ex` render entry points. */
enum {
  /* Run the reference's every-shape loop (world.rs:31-38) instead of the
   * exact-culling fast path: same image bit for bit, every counter exact
   * (incl. sphere_disc_ge0), ~15x slower. For parity checks and counting. */
  RT_RENDER_EXHAUSTIVE = 1
};

typedef struct rt_scene rt_scene; /* opaque: device-resident flattened World */

/* ---- host math helpers (exact restatements used to build descs) --------- */

/* `Matrix::inverse` (matrix.rs:138-153) by cofactor expansion, bit-exact.
 * Returns RT_ERR_NOT_INVERTIBLE when |det| < 1e-5 (matrix.rs:134-136). */
int rt_matrix_inverse(const double m[16], double out[16]);

/* `Camera::new` (camera.rs:33-55) + `Camera::set_transform` (camera.rs:128-131). */
int rt_camera_init(uint32_t hsize, uint32_t vsize, double field_of_view,
                   const double transform[16], rt_camera_desc* out);

/* ---- scene lifetime ------------------------------------------------------ */

/* Flatten + upload a World (replaces building `World` for `Camera::render`).
 * `device` is the HIP ordinal. Fails with RT_ERR_DUPLICATE_SHAPES when two
 * shapes may be structurally equal (the refractive-index `containers` walk,
 * geometry/intersection.rs:63-90, then depends on structural equality). */
int rt_scene_create(const rt_shape_desc* shapes, size_t n_shapes,
                    const rt_light_desc* lights, size_t n_lights, int device,
                    rt_scene** out);

/* (ABI 6) rt_scene_create for a World whose objects include Groups
 * (group.rs): `shapes` are the primitives in the order World::intersect's
 * flat_map reaches them (each group's children in order, depth first), with
 * their final transforms (the groups' transforms baked in, group.rs:71-94,
 * 128-133) and materials (Group::set_material, :96-102); shape_group[i] is the
 * innermost group of shape i (-1: none). A shape inside groups is intersected
 * only by rays that meet the box of every group around it
 * (BoundingBox::intersects, bounding_box.rs:95-136, its |d| < EPSILON rule
 * included), exactly as the reference's Group::intersect skips its children. */
int rt_scene_create_groups(const rt_shape_desc* shapes, size_t n_shapes,
                           const int32_t* shape_group, const rt_group_desc* groups,
                           size_t n_groups, const rt_light_desc* lights,
                           size_t n_lights, int device, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);

/* ---- render entry points -------------------------------------------------- */

/* `Camera::render(&mut self, &World) -> Canvas` (camera.rs:133-148) with
 * `MAX_RECURSION_DEPTH` replaced by `max_depth` (world.rs:16; 5 = reference).
 * `out_rgb` is a caller-owned HOST buffer of vsize*hsize*3 doubles, row-major
 * `y*w + x` (canvas.rs:44-48). Synchronous. A large frame (>= 2^20 samples)
 * without `stats` is rendered in row bands on the call's own streams, each
 * band's copy to `out_rgb` running behind its render while the next bands
 * render; the pixels are the whole-frame render's. The copy goes straight into
 * `out_rgb` by DMA when it comes from rt_host_buffer_alloc (the fast case),
 * else the buffer is page-locked for the call. */
int rt_render(const rt_scene* scene, const rt_camera_desc* camera,
              uint32_t max_depth, double* out_rgb, rt_stats* stats);

/* `Camera::render_multithreaded` (camera.rs:150-214): every pixel is the
 * `Color::average` (color.rs:26-33) of `color_at` over the rays of
 * `rays_for_pixel` (camera.rs:71-126) for `aa_samples` in {1,2,4,8,16}
 * (`RenderOpts::aa_samples`). The reference's `num_threads` only partitions
 * CPU work and does not change the image. aa_samples == 1 equals rt_render. */
int rt_render_aa(const rt_scene* scene, const rt_camera_desc* camera,
                 uint32_t max_depth, uint32_t aa_samples, double* out_rgb,
                 rt_stats* stats);

/* rt_render_aa with `flags` (RT_RENDER_*). */
int rt_render_ex(const rt_scene* scene, const rt_camera_desc* camera,
                 uint32_t max_depth, uint32_t aa_samples, uint32_t flags,
                 double* out_rgb, rt_stats* stats);

/* Device-resident shard render (used by multi-GPU and the benchmark).
 * Renders the rows y with (y / row_block) % n_shards == shard, in increasing
 * y order, into `d_out_rgb` (a DEVICE buffer on the scene's device holding
 * rows_in_shard*hsize*3 doubles). `stream` is a hipStream_t; NULL means the
 * default (null) stream, so the work is ordered with the caller's other work
 * there (torch's current stream is often the null stream).
 * Asynchronous unless `stats` is non-NULL (then it synchronises to read the
 * counters): the host enqueues the whole frame without waiting, whatever the
 * camera. `n_shards == 1` renders the whole frame. `aa_samples` as in
 * rt_render_aa (1 = `Camera::render`).
 * Deferred errors: an asynchronous call returns before its frame has run, so
 * a device-side failure of that frame (see rt_scene_check) is reported by the
 * next call on the scene, or by rt_scene_check. */
int rt_render_shard_device(const rt_scene* scene, const rt_camera_desc* camera,
                           uint32_t max_depth, uint32_t aa_samples,
                           uint32_t row_block,
                           uint32_t shard, uint32_t n_shards,
                           double* d_out_rgb, void* stream, rt_stats* stats);

/* rt_render_shard_device with `flags` (RT_RENDER_*). */
int rt_render_shard_device_ex(const rt_scene* scene, const rt_camera_desc* camera,
                              uint32_t max_depth, uint32_t aa_samples,
                              uint32_t row_block, uint32_t shard, uint32_t n_shards,
                              uint32_t flags, double* d_out_rgb, void* stream,
                              rt_stats* stats);

/* `Camera::render` (camera.rs:133-148) of `n_frames` cameras sharing hsize and
 * vsize (the frames of an animation, or the steady state of a frame loop)
 * over the same world: frame f's shard (as rt_render_shard_device) goes to the
 * DEVICE buffer d_out_rgb[f]. Each frame equals its rt_render_shard_device
 * render bit for bit; the frames are rendered together, up to 16 per pass of
 * the pipeline and at most 2^25 root rays (pixels x aa_samples) per pass (one
 * launch per recursion generation carries all of them), so
 * small frames and shards pay the per-pass cost once. Asynchronous on
 * `stream` unless `stats` is non-NULL: then the frames are rendered one by
 * one and the counters summed over them. Deferred errors as
 * rt_render_shard_device. */
int rt_render_frames_device(const rt_scene* scene, const rt_camera_desc* cameras,
                            uint32_t n_frames, uint32_t max_depth,
                            uint32_t aa_samples, uint32_t row_block,
                            uint32_t shard, uint32_t n_shards,
                            double* const* d_out_rgb, void* stream,
                            rt_stats* stats);

/* Number of rows shard `shard` of `n_shards` owns (for sizing buffers). */
uint32_t rt_shard_rows(uint32_t vsize, uint32_t row_block, uint32_t shard,
                       uint32_t n_shards);

/* (ABI 6) rt_render_frames_device over a block PATTERN instead of an
 * interleaved shard: the canvas's row blocks (row_block rows each) are dealt
 * in periods of `period` blocks (1..64), and this render owns the blocks whose
 * position in their period is a set bit of `mask` (non-zero, below
 * 2^period). Its rows go to d_out_rgb[f] in increasing y order. A shard
 * (shard s of n) is the pattern (period n, mask 1 << s); uneven patterns let a
 * multi-GPU caller give one rank fewer rows than the others (the rank that
 * also assembles the canvas; rtamd.distributed.block_patterns), as the
 * reference's render_multithreaded gives its last thread the remainder
 * (camera.rs:157-172). `flags`: RT_RENDER_*. Asynchronous and deferred errors
 * as rt_render_frames_device. */
int rt_render_block_pattern_device(const rt_scene* scene, const rt_camera_desc* cameras,
                                   uint32_t n_frames, uint32_t max_depth,
                                   uint32_t aa_samples, uint32_t row_block,
                                   uint32_t period, uint64_t mask, uint32_t flags,
                                   double* const* d_out_rgb, void* stream,
                                   rt_stats* stats);

/* (ABI 6) Number of rows a block pattern owns (0 for an invalid pattern). */
uint32_t rt_pattern_rows(uint32_t vsize, uint32_t row_block, uint32_t period,
                         uint64_t mask);

/* `World::color_at(&Ray, remaining)` (world.rs:70-81) for a batch of rays.
 * rays: n*6 doubles (origin xyz, direction xyz); out_rgb: n*3 doubles (host). */
int rt_color_at_batch(const rt_scene* scene, const double* rays, size_t n,
                      uint32_t remaining, double* out_rgb, rt_stats* stats);

/* rt_color_at_batch with `flags` (RT_RENDER_*). */
int rt_color_at_batch_ex(const rt_scene* scene, const double* rays, size_t n,
                         uint32_t remaining, uint32_t flags, double* out_rgb,
                         rt_stats* stats);

/* `World::is_shadowed(point, light)` (world.rs:95-105) for a batch of points
 * against light index `light`. out: n uint8 (1 = shadowed). */
int rt_is_shadowed_batch(const rt_scene* scene, const double* points, size_t n,
                         uint32_t light, uint8_t* out);

/* `World::intersect` + `hit` + `prepare_computations` + `schlick`
 * (world.rs:31-38, intersection.rs:53-105,118-120,147-162) for a batch of
 * rays. Per ray, out holds 24 doubles:
 *   [0] hit object index (-1 = miss)  [1] t   [2..4] point
 *   [5..7] over_point  [8..10] under_point  [11..13] eyev  [14..16] normalv
 *   [17] inside (0/1)  [18..20] reflectv  [21] n1  [22] n2  [23] schlick */
int rt_hit_batch(const rt_scene* scene, const double* rays, size_t n,
                 double* out24);

/* ---- multi-GPU (one process, several devices; the per-process path for
 *      torch.distributed is rt_render_shard_device) ------------------------ */

/* `Camera::render_multithreaded` across devices (camera.rs:150-217): render on
 * `n_devices` devices (ordinals 0..n-1) with interleaved blocks of `row_block`
 * rows (block b on device b mod n; the reference's row-block partition,
 * camera.rs:157-172). Output to a HOST buffer like rt_render: each device's
 * DMA engine copies its rows straight into the canvas over its own link, each
 * device driven by its own host thread; one device renders as rt_render does.
 * The canvas is registered for the call unless it is a pinned block
 * (rt_host_buffer_alloc) or pinned by the caller. `scenes[i]` must have been
 * created on device i. Development knob `multi_gather` (scene 0): every shard
 * gathered into device 0 with one grouped RCCL ncclGather instead. */
int rt_render_multi(rt_scene* const* scenes, int n_devices,
                    const rt_camera_desc* camera, uint32_t max_depth,
                    uint32_t aa_samples, uint32_t row_block, double* out_rgb,
                    rt_stats* stats);

/* ---- output (image/ppm.rs) ------------------------------------------------ */

/* `canvas_to_ppm` (image/ppm.rs:24-51): plain P3 text, 70-column wrapping,
 * `(v*255).round() as u8` quantisation. If out == NULL or cap too small,
 * *out_len receives the required size and RT_ERR_BUFFER_TOO_SMALL (or RT_OK
 * with out == NULL) is returned. No terminating NUL is written. */
int rt_canvas_to_ppm(const double* rgb, uint32_t width, uint32_t height,
                     char* out, size_t cap, size_t* out_len);

/* `canvas_to_ppm` (image/ppm.rs:24-51) of a DEVICE canvas (rows x width x 3
 * f64, row-major, as rt_render_shard_device writes it) into DEVICE memory
 * `d_out` (cap bytes), on `stream` (NULL = the default stream). The bytes are
 * those rt_canvas_to_ppm writes. *out_len receives the text's length (d_out ==
 * NULL: the length only); a buffer of 12 * width * height + height + 32 bytes
 * always suffices. Returns after the text is complete. width <= 12288. */
int rt_canvas_to_ppm_device(const double* d_rgb, uint32_t width, uint32_t height,
                            char* d_out, size_t cap, size_t* out_len, void* stream);

/* `canvas_to_ppm(&camera.render(&world))` (camera.rs:133-148 then
 * image/ppm.rs:24-51; the render_scene / demo-binary output path) in one call:
 * the frame is rendered, encoded on the device and only the PPM text crosses
 * to the host buffer `out` (cap bytes). *out_len receives the text's length;
 * out == NULL asks for the length only (the frame is still rendered), and a
 * too-small cap returns RT_ERR_BUFFER_TOO_SMALL. hsize <= 12288. */
int rt_render_ppm(const rt_scene* scene, const rt_camera_desc* camera,
                  uint32_t max_depth, uint32_t aa_samples, char* out, size_t cap,
                  size_t* out_len, rt_stats* stats);

/* `scale_color_component` (image/ppm.rs:73-75) over n values. */
int rt_quantize_u8(const double* values, size_t n, uint8_t* out);

/* ---- host buffers ------------------------------------------------------------ */

/* Page-locked host memory for the outputs of the host-buffer entry points
 * (rt_render, rt_render_aa, rt_render_ex, rt_color_at_batch, ...): the device
 * writes such a buffer directly at the full link rate, where a pageable buffer
 * is pinned for the duration of each call (or staged). A Canvas that lives for
 * many frames (or a pool of them) keeps its pixels here. Released blocks are
 * pooled (up to 1 GiB) and handed out again for requests of about their size.
 * NULL on failure (rt_last_error). */
void* rt_host_buffer_alloc(size_t bytes);
void rt_host_buffer_free(void* p);

/* ---- diagnostics ----------------------------------------------------------- */
const char* rt_last_error(void);
int rt_abi_version(void);
int rt_device_count(void);

/* Sizes of the ABI structs as this library was built (ABI 6). A foreign
 * binding (INTEGRATION.md's Rust `#[repr(C)]` mirrors) asserts its own
 * `size_of` against these before its first call: rt_stats is filled in full
 * (sizeof(rt_stats) bytes) by every entry point that takes one. */
size_t rt_sizeof_shape_desc(void);  /* 680 */
size_t rt_sizeof_camera_desc(void); /* 160 */
size_t rt_sizeof_stats(void);       /* 112 */

/* Waits for every render issued on `scene` (on any stream) and reports any
 * frame the library found incomplete after the fact. The wavefront queues of
 * an asynchronous render live in per-workspace arenas sized from the frames
 * the scene has rendered (DESIGN.md "Device-sized generations"); a frame
 * whose recursion outgrows them is detected on the device, left incomplete,
 * and reported as RT_ERR_HIP by the NEXT call on the scene, or by this one,
 * after the arenas have grown (render that frame again). Such a frame never
 * looks valid: every pixel of its canvas (of every canvas of its batch) is
 * NaN. Synchronous calls never report it: they grow the arenas and render
 * again themselves. Until a scene has rendered a frame, the arenas are sized
 * from default ratios, so a first asynchronous frame of a deeply recursive
 * scene may be one of these. Callers
 * that render asynchronously call it after their last frame to learn about
 * every frame. RT_OK when all frames were complete. */
int rt_scene_check(const rt_scene* scene);

#ifdef __cplusplus
}
#endif
#endif /* RT_RENDER_H */
