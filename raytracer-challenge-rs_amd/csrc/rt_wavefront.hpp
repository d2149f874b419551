// rt_wavefront.hpp — host side of the wavefront render pipeline.
//
// The recursion tree of `World::color_at` (world.rs:70-81) is evaluated one
// GENERATION (recursion depth) at a time over flat ray queues.
//
// Fast path (BVH; DESIGN.md "Fused generations"), one launch per generation:
//   for g = 0 .. max_depth:
//     trace_fused(g)   World::intersect + hit, prepare_computations, the
//                      reflected / refracted children -> rays_{g+1}, every
//                      light's is_shadowed + lighting (world.rs:40-56), and
//                      the final colour of each node without children
//                      -> colors_g; nodes with children -> parents_g
//   for g = max_depth .. 0:
//     combine_parents(g)  shade_hit's sum with the children's colours
//                         (world.rs:58-67)                     -> colors_g
//
// Exhaustive pipeline (the reference's every-shape loop; counted launches):
//   for g = 0 .. max_depth:
//     trace_closest(g)  World::intersect + hit          -> hits_g
//     prep(g)           prepare_computations; spawn the shadow rays
//                       (is_shadowed, world.rs:95-105) and the reflected /
//                       refracted children (world.rs:107-134)   -> nodes_g,
//                       shadow queue S_g, rays_{g+1}
//     trace_shadow(g)   any-hit test of S_g + lighting()        -> surf_g
//   for g = max_depth .. 0:
//     combine(g)        lighting over lights (left fold) + children colours,
//                       Schlick or plain sum (world.rs:40-68)   -> colors_g
//
// Every node's colour is computed from its children's colours with exactly
// the reference's expression, so the result equals the recursive evaluation
// bit for bit (no path-weight re-association). Queue order does not affect
// any value.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "rt_layout.hpp"

namespace rtamd {

// Sharded generation queues (DESIGN.md "Sharded queues"): kShards regions per
// queue, counters kShardStride uints (128 B) apart.
constexpr int kShards = 64;
constexpr int kShardStride = 32;
constexpr int kShardGroup = 16;  // consecutive wave-iterations sharing a region (one block's worth)

struct alignas(16) WfRay {  // 48 B: three 16-B loads / stores per ray
  double o[3];
  double d[3];
};
static_assert(sizeof(WfRay) == 48, "WfRay is origin + direction only");
struct WfHit {  // 24 B: nearest hit + containers top-2 (rt_device.hpp Hit)
  double t;
  int32_t key, c1k, c2k, hin;
};
struct WfNode {  // 24 B: what shade_hit needs besides the lighting (which prep_one evaluates)
  double schlick;      // Computations::schlick (only read when reflective && transparent)
  int32_t obj;         // -1 = miss
  int32_t child_refl;  // index into rays_{g+1}, -1 = none (black)
  int32_t child_refr;
  int32_t pad;
};
// A fast-path node with children (48 B): its surface term (the lighting sum
// over the lights), Schlick factor, colour slot and children (wf_combine_parents).
struct ParentRec {
  double surface[3];
  double schlick;      // Computations::schlick (only read when reflective && transparent)
  uint32_t slot;       // the node's slot in generation g (its colour's place)
  int32_t obj;
  int32_t child_refl;  // index into rays_{g+1}, -1 = none (black)
  int32_t child_refr;
};
struct PrimRec {  // primary rays share the origin: per diag sphere (s, o', c)
  double s[3];
  double op[3];
  double c;
  double pad;
};

constexpr int kMaxGen = 66;
// LDS a fused trace launch may take (of the CU's 160 KB)
constexpr size_t kFusedLdsLimit = 160 * 1024 - 1024;
constexpr int kFusedBlockThreads = 1024;  // threads of a fused trace block (kTraceBlock, rt_trace.hpp)
enum WfFlags : unsigned { WF_EXHAUSTIVE = 1u, WF_COUNT = 2u, WF_TIME = 4u };  // WF_TIME: events around the render (kernel_ms)

// Render-time tuning of a scene (rt_scene::tune, copied from the process
// defaults when the scene is created; rtamd_scene_tuning_set changes one
// scene's). Every render reads its scene's values under the scene's lock, so
// concurrent renders of different scenes never see each other's settings.
struct WfTuning {
  int accel = 1;           // 1 = exact-culling BVH fast path (unless the exhaustive loop is asked for)
  int skip_shadow = 1;     // 1 = the fast path leaves out shadow rays that cannot change the colour
  int shadow_lb = 1;       // 1 = shadow rays through the light buffer when the scene has one
  int image = 0;           // 0 = automatic scene image of the fast-path kernels, 3 / 1 = global memory
  int treelet = 1;         // the global-memory image stages a treelet in LDS
  int wide = 1;            // the global-memory image: 1 = the four-wide hierarchy (BvhWide) when the scene has one
  int lds_wide = 1;        // fast path: 1 = the four-wide hierarchy and 48-B records in LDS (LANE 15) when they fit
  int treelet_deltas = 1;  // ... after the light buffer's distances (when they fit)
  int shadow_stream = 1;   // exhaustive pipeline: 1 = shadow traces on a second stream when rendering alone
  int adaptive_block = 0;  // generation pipeline: 1 = small trace launches spread over every CU
  int prim_lane = 1;       // fast path: primary rays by the per-lane walk instead of the wave traversal with
                           //     shared-origin records: 1 = over any image (default), 2 = over the LDS images only, 0 = never
  int arena_pct = 100;     // test hook: the fast path's queue arenas sized to this percentage of the hint,
                           //     shrinking them (< 100: forces overflows, DESIGN.md "Device-sized generations")
  int d2h = 1;             // host-canvas copies: 1 = pin the caller's buffer for the call and DMA into it, 0 = pinned chunks
  int bands = 4;           // rt_render into a host canvas: row bands rendered one after the other on their own
                           //     streams, each band's device-to-host copy overlapping the next bands' renders (1 = one
                           //     render, then one copy)
  int band_pct = 35;       // ... the first band's share of the rows (percent)
  int band_ratio = 100;    // ... each later band's size, percent of the one before (100: equal shares)
  int band_gen = 1;        // ... band k+1 starts when band k's generation band_gen has run (-1: its whole render)
  int multi_gather = 0;    // rt_render_multi (scenes[0]'s knob): 1 = every shard gathered into device 0 by one grouped
                           //     ncclGather, then copied out of device 0 (test hook; 0 = each device copies its rows
                           //     straight into the host canvas, rt_multi.cpp)
  int spread = 0;          // fast path: 1 = a launch with fewer 64-ray chunks than waves deals its chunks round-robin
                           //     over its blocks (every CU) instead of filling the first blocks: a small frame rendered
                           //     alone 24-29 % faster, but frames in flight lose (8-way shards +23 %, banded rt_render
                           //     +4 %: the blocks then hold every CU's LDS with a few waves each), so not the default
  int own_sphere = 2;      // fast path, the shadow rays of a hit on a sphere record: 1 = from inside, test that sphere
                           //     first; 2 = also, from outside towards a light in front, leave it out (rt_trace.hpp)
};
// Applies `key` = `value` to `t`: 1 = applied, 0 = not a render-time key, -1 = bad value.
int wf_tuning_apply(WfTuning& t, const char* key, int value);

// The fast path's launch over a global-memory scene image (lane 3 or 1) of
// one generation: compiled into its own code object (rt_wavefront.hip built
// with -DRT_WF_GLOBAL_TU). e0/e1: launch-carried profiling events, or null.
struct DevCamera;
struct WfArgs;
hipError_t wf_launch_global(int lane, bool quads, bool tally, bool cam_rays, const DevScene& sc, const DevCamera& cam,
                            const WfArgs& a, size_t dyn, unsigned n, hipStream_t stream, int block, hipEvent_t e0,
                            hipEvent_t e1);

// Work counters of the trace kernels, one row per wave slot (wave id mod
// kWorkRows, rows 128 B apart): thousands of waves ending together would
// otherwise queue on one address (one L2 atomic at a time), which cost the
// short light-buffer launches most of their time. The host sums the rows.
constexpr int kWorkRows = 256;
struct alignas(128) WfWorkRow {
  unsigned long long disc[3];   // disc >= 0 tests: [0] primary closest, [1] closest, [2] shadow
  unsigned long long tests[3];  // BVH mode: sphere tests executed (lanes x spheres), per trace class
  unsigned long long boxes[3];  // BVH mode: child-box tests executed (lanes x boxes)
  unsigned long long sh_rays[2];   // fused kernels: shadow rays traced, [0] primary / [1] secondary launches
  unsigned long long sh_tests[2];  // fused kernels: shadow sphere tests executed, per launch class
  unsigned long long gated[3];     // shapes a group's box kept out of a ray: spheres, planes, others (GateSkips)
};
// Fused launches hand out their rays in chunks of 64 (one wave-iteration) from
// per-XCD counters, kChunkClasses per generation, each on a 128-B line.
constexpr int kChunkClasses = 8;
constexpr int kChunkStride = 32;
struct WfCounters {
  unsigned chunk[kMaxGen * kChunkClasses * kChunkStride];
  unsigned n_refl[kMaxGen], n_refr[kMaxGen], n_hit[kMaxGen];
  // this pass (frame or batch) outgrew its arenas (bind_generation): its
  // canvases are filled with NaN by the last launch (poison_frames)
  unsigned overflow;
  WfWorkRow work[kWorkRows];
  unsigned long long disc(int c) const {
    unsigned long long t = 0;
    for (int r = 0; r < kWorkRows; ++r) t += work[r].disc[c];
    return t;
  }
  unsigned long long tests(int c) const {
    unsigned long long t = 0;
    for (int r = 0; r < kWorkRows; ++r) t += work[r].tests[c];
    return t;
  }
  unsigned long long boxes(int c) const {
    unsigned long long t = 0;
    for (int r = 0; r < kWorkRows; ++r) t += work[r].boxes[c];
    return t;
  }
  unsigned long long sh_rays(int c) const {
    unsigned long long t = 0;
    for (int r = 0; r < kWorkRows; ++r) t += work[r].sh_rays[c];
    return t;
  }
  unsigned long long sh_tests(int c) const {
    unsigned long long t = 0;
    for (int r = 0; r < kWorkRows; ++r) t += work[r].sh_tests[c];
    return t;
  }
  unsigned long long gated(int c) const {
    unsigned long long t = 0;
    for (int r = 0; r < kWorkRows; ++r) t += work[r].gated[c];
    return t;
  }
};

struct WfGeo {  // 80 B: the lighting() inputs of a hit (comps.over_point, normalv, eyev)
  double over[3], normal[3], eyev[3];
  int32_t obj;
  int32_t pad;
};
struct WfGenBuf {  // grow-only, the exhaustive pipeline's per-generation arrays
  WfRay* rays = nullptr;
  double* colors = nullptr;
  WfHit* hits = nullptr;
  WfNode* nodes = nullptr;
  int32_t* shadow_nodes = nullptr;  // shadow list of the generation (node slot * L + light, sharded)
  WfGeo* geo = nullptr;              // per node slot: what the shadow trace needs to evaluate lighting()
  double* surf = nullptr;            // lighting() per node slot and light (3 doubles)
  size_t cap_rays = 0, cap_colors = 0, cap_hits = 0, cap_nodes = 0, cap_list = 0, cap_geo = 0, cap_surf = 0;
};

// Device-sized generations (the fast path; DESIGN.md "Device-sized
// generations"). The host never learns a generation's ray count before its
// launch: the launch of generation g reads it from the queue counters, sizes
// the sharded regions of generation g+1 and of its own parent list from it,
// and places them in three per-workspace arenas (colours, parent records, and
// two ping-pong ray buffers). Generation g's place, written by generation
// g-1's launch (g = 0: by wf_frame_init):
struct WfGenTab {
  unsigned cap;                   // per-region capacity of its rays / colours (0: generation 0, dense)
  unsigned pad;
  unsigned long long color_off;   // its first colour slot in the colour arena
  unsigned long long par_off;     // its parent list's first record in the parent arena
};
// A generation that does not fit the arenas spawns no children (the frame is
// then incomplete): its launch raises `overflow` in this host-mapped record of
// the workspace with what it needed. Every frame's last combine also records
// the frame's ray count per generation, from which the host sizes the arenas
// of later frames (WfSizing); nothing waits for it.
struct WfHostRec {
  int overflow;
  int pad[3];
  unsigned long long need_colors, need_parents, need_rays;  // of the generation that overflowed
  unsigned long long frames;   // frames recorded (the counts below are the last one's)
  unsigned n_real;             // root rays (without the padding of a batch)
  unsigned n_gens;             // generations counted (max_depth + 1)
  unsigned counts[kMaxGen];    // rays of each generation
};
// Arena sizes learned per scene (every workspace of a scene reads and
// updates them under the scene's lock): per root ray, the most secondary
// work any frame needed (rho = sum of the ray counts of the generations that
// may spawn children / root rays; mu = largest generation / root rays).
struct WfSizing {
  double rho = 0.0, mu = 0.0;
  int branch = 2;  // children per ray at most: 0 no reflective or transparent material, 1 never both, 2 otherwise
};

// A batch of frames rendered by one pass of the generation pipeline (camera
// mode): every generation's launch carries the rays of all of them, so a
// small frame (a multi-GPU shard) still fills the GPU and the chain of
// dependent launches is paid once per batch. Frame f's root rays are slots
// [f * frame_rays, f * frame_rays + frame_real) of generation 0 (frame_rays
// padded to whole 64-ray chunks, so a chunk never mixes two cameras).
constexpr unsigned kMaxFrames = 16;
struct FrameTable {
  DevCamera cam[kMaxFrames];
  double* out[kMaxFrames];  // device canvases (the shard's rows, row-major)
};

// Kernel arguments for one generation.
struct WfArgs {
  WfRay* rays;          // rays_g (g >= 1 or batch mode)
  WfHit* hits;
  WfNode* nodes;
  double* colors;       // colors_g (g >= 1) or the output (g == 0)
  int32_t* shadow_nodes;  // shadow list of this generation: entries node slot * L + light
  WfGeo* geo;           // per node slot: over point, normal, eye vector, object
  double* surf;         // per node slot * L + light: lighting() (written by prep_one when the light needs
                        // no shadow ray, else by the shadow trace)
  ParentRec* parents;   // fast path: this generation's nodes with children (sharded like the shadow list)
  WfRay* next_rays;     // rays_{g+1}
  const double* child_colors;  // colors_{g+1}
  WfCounters* cnt;
  const PrimRec* prim;  // per-frame primary records (camera mode, g == 0)
  unsigned n;           // rays in this generation
  unsigned n_shadow;    // shadow rays in this generation
  unsigned g, max_depth;
  unsigned camera_mode; // g == 0 rays come from the camera (1) or from `rays` (0)
  unsigned row_block, shard, n_shards;
  // a block-pattern render (rt_render_block_pattern_device): the canvas's row
  // blocks are dealt in periods of blk_period blocks, of which this render owns
  // the positions set in blk_mask; its local block i is canvas block
  // (i / popcount(mask)) * period + the (i mod popcount(mask))-th set bit.
  // blk_period 0: the interleaved shard (block b -> shard b mod n_shards).
  unsigned long long blk_mask;
  unsigned blk_period;
  unsigned disc_slot;   // WfCounters::disc index of this trace launch
  unsigned aa;          // AA samples per pixel (generation 0 in camera mode)
  unsigned rows;        // local rows of the camera shard (generation-0 tiling)
  unsigned skip_shadow; // leave out shadow rays that cannot change the colour (fast path)
  unsigned own_sphere;    // fast path: WfTuning::own_sphere
  unsigned spread;        // fast path: WfTuning::spread (a launch of fewer chunks than waves deals them over the blocks)
  // sharded queues: this generation's rays (in_cnt == nullptr: dense, slot = index),
  // the next generation's rays and this generation's shadow list
  const unsigned* in_cnt;
  unsigned in_cap;      // per-region capacity of this generation's arrays
  unsigned* out_cnt;
  unsigned out_cap;     // per-region capacity of the next generation's arrays
  unsigned* sh_cnt;
  unsigned sh_cap;      // per-region capacity of the shadow list (fast path: of the parents)
  unsigned count;       // counted launch: tally shade_hit runs and children (fast path)
  unsigned use_lb;      // fast path: shadow rays through the light buffer
  unsigned lds_flags;   // fast path: what the trace kernel stages in LDS (kLdsSpheres | kLdsDeltas)
  unsigned n_top;       // fast path, global-memory image: the first n_top (breadth-first) nodes are in LDS
  unsigned n_frames;    // camera mode: frames in this pass (1: cam / colors; > 1: `frames`)
  unsigned frame_rays, frame_real;  // n_frames > 1: generation-0 slots per frame, root rays per frame
  const FrameTable* frames;         // n_frames > 1: the device copy of the batch's cameras and canvases
  // device-sized generations (fast path): bind_generation fills n, in_cap,
  // out_cap, sh_cap, rays, next_rays, colors and parents from the tables
  unsigned dev_sized;
  unsigned colors_direct;           // generation 0's colours go to `colors` as given (the output)
  WfGenTab* gtab;                   // [kMaxGen + 1]
  unsigned* gsh;                    // [kMaxGen]: per-region capacity of generation g's parent list
  WfRay* ray_buf[2];                // generation g's rays in ray_buf[g & 1]
  double* color_base;
  ParentRec* par_base;
  unsigned long long color_cap, par_cap, ray_cap;  // colour slots, parent records, ray slots per buffer
  WfHostRec* hrec;                  // device address of the workspace's host-mapped record
};

// Per-kernel-class timing of the last frame (profiling mode only).
enum WfClass { WF_PRIMARY = 0, WF_CLOSEST = 1, WF_SHADOW = 2, WF_PREP = 3, WF_COMBINE = 4, WF_NCLASS = 5 };
struct WfProfile {
  double ms[WF_NCLASS];
  double rays[3];   // rays traced by the three trace classes
  double disc[3];   // disc >= 0 tests per trace class
  double tests[3];  // sphere tests executed per trace class (exhaustive: rays x n_diag)
  double boxes[3];  // BVH child-box tests executed per trace class (0 when exhaustive)
  double sh_rays[2], sh_tests[2];  // fused frames: shadow rays / sphere tests inside the primary / secondary launches
  int bvh;          // the last frame traversed the BVH
  int fused;        // the last frame ran the fused pipeline
};

class Wavefront {
 public:
  ~Wavefront();
  // Profiling mode: start/stop events carried by every launch of the kernel
  // classes in `class_mask` (bit WF_*), summed per class.
  void set_profiling(bool on, int class_mask = (1 << WF_NCLASS) - 1) {
    profiling_ = on;
    pmask_ = class_mask;
    if (on) { pn_ = 0; pframes_ = 0; }
  }
  size_t profiled_frames() const { return pframes_; }
  // Per-class times averaged over the frames rendered since profiling was
  // enabled; rays / disc counts of the last frame (synchronises).
  hipError_t last_profile(WfProfile* out);
  // Render n0 root rays (camera pixels x `aa` samples of a shard, or explicit
  // rays) into `out` (n0/aa*3 doubles, device; AA samples are averaged like
  // Color::average). The fast path (BVH) is fully asynchronous: every
  // generation sizes itself on the device (WfGenTab); `sz` sizes the arenas.
  // The exhaustive pipeline (WF_EXHAUSTIVE or a scene without hierarchies)
  // reads each generation's count back (synchronous). stats (host) may be
  // null. `solo`: no other workspace renders concurrently (then the
  // exhaustive shadow traces take the side stream).
  // `flags`: WF_EXHAUSTIVE runs the reference's every-shape loop (exact
  // sphere_disc_ge0); WF_COUNT counts the reference's rays of this render
  // (read later by read_stats). A non-null `stats` implies WF_COUNT and
  // synchronises to fill it.
  // `blk_period` / `blk_mask`: a block-pattern render (WfArgs::blk_mask) instead of
  // shard `shard` of `n_shards` (blk_period 0).
  hipError_t render(const DevScene& sc, const DevCamera& cam, bool camera_mode, const double* d_in_rays,
                    unsigned n0, unsigned aa, unsigned max_depth, unsigned row_block, unsigned shard,
                    unsigned n_shards, double* d_out, hipStream_t stream, WfSizing& sz, DevStats* stats,
                    float* ms_kernel, const WfTuning& tn, bool solo = true, unsigned flags = 0,
                    const FrameTable* batch = nullptr, unsigned n_frames = 1, unsigned blk_period = 0,
                    unsigned long long blk_mask = 0);
  // The counters of the last render (rendered with WF_COUNT); synchronises its stream.
  hipError_t read_stats(DevStats* out);
  // Rays of each generation of the last render (synchronises its stream).
  hipError_t gen_counts(std::vector<unsigned>& rays) { return last_counts(rays); }
  // Device time of the last render rendered with WF_TIME (after it completed).
  hipError_t kernel_ms(float* ms) { return hipEventElapsedTime(ms, ev0_, ev1_); }
  // A fast-path frame of this workspace overflowed its arenas (WfHostRec):
  // that frame is incomplete. take_overflow() clears the flag and grows the
  // arenas past what the overflowing generation asked for (the next frame
  // fits at least that generation); it returns whether the flag was set.
  // Call it only once the frame has completed (after a synchronisation).
  bool overflowed() const { return h_rec_ && ((volatile WfHostRec*)h_rec_)->overflow != 0; }
  hipError_t take_overflow(bool* was);
  // The learned sizes from this workspace's last recorded frame (non-blocking:
  // the record of a frame still in flight may be stale).
  void learn(WfSizing& sz) const;
  // The next fast-path render records `ev` on its stream right after the launch
  // of generation g (rt_render's bands: the next band may start while this one's
  // deeper, smaller generations run); gen_event_recorded() tells whether it did
  // (a render with fewer generations, or an exhaustive one, does not).
  void set_gen_event(hipEvent_t ev, int g) { gen_ev_ = ev; gen_ev_g_ = g; gen_ev_done_ = false; }
  bool gen_event_recorded() const { return gen_ev_done_; }

 private:
  hipError_t render_fast(const DevScene& sc, const DevCamera& cam, bool camera_mode, const double* d_in_rays,
                         unsigned n0, unsigned frame_real, unsigned aa, unsigned max_depth, unsigned row_block,
                         unsigned shard, unsigned n_shards, double* d_out, hipStream_t stream, WfSizing& sz,
                         bool count, bool skip_shadow, const WfTuning& tn, const FrameTable* batch,
                         unsigned n_frames);
  hipError_t render_exhaustive(const DevScene& sc, const DevCamera& cam, bool camera_mode, const double* d_in_rays,
                               unsigned n0, unsigned aa, unsigned max_depth, unsigned row_block, unsigned shard,
                               unsigned n_shards, double* d_out, hipStream_t stream, bool count, bool skip_shadow,
                               const WfTuning& tn, bool solo);
  hipError_t ensure_gen(size_t g, size_t slots, size_t n_lights, size_t list_slots);
  hipError_t ensure_misc(size_t n_diag, unsigned n_frames = 1);
  hipError_t ensure_arenas(unsigned long long colors, unsigned long long parents, unsigned long long rays,
                           bool exact);
  // shard counters: generation g's rays (q = 0) / shadow list (q = 1)
  unsigned* shard_cnt(unsigned g, unsigned q) { return d_shard_ + ((size_t)g * 2 + q) * kShards * kShardStride; }
  std::vector<WfGenBuf> gens_;
  // the fast path's arenas (grow-only; arena_pct < 100 shrinks them, a test hook)
  double* colors_ = nullptr;
  ParentRec* parents_ = nullptr;
  WfRay* rays_[2] = {nullptr, nullptr};
  unsigned long long color_cap_ = 0, par_cap_ = 0, ray_cap_ = 0;
  int squeezed_pct_ = 100;  // the arena_pct the arenas were last shrunk to
  WfGenTab* d_gtab_ = nullptr;
  unsigned* d_gsh_ = nullptr;
  WfHostRec* h_rec_ = nullptr;  // host-mapped (hipHostMallocMapped)
  WfHostRec* d_rec_ = nullptr;  // its device address
  WfCounters* d_cnt_ = nullptr;
  unsigned* d_shard_ = nullptr;  // kMaxGen x 2 x kShards counters, kShardStride apart
  PrimRec* d_prim_ = nullptr;
  size_t prim_cap_ = 0;
  FrameTable* d_frames_ = nullptr;  // the current batch's table (written by wf_frame_init)
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  // shadow traces run on a second stream (DESIGN.md "Shadow stream"): fork
  // event per generation (recorded after its closest-hit launch), one join
  hipStream_t side_ = nullptr;
  int side_dev_ = -1;
  hipEvent_t fork_ev_[kMaxGen] = {};
  hipEvent_t join_ev_ = nullptr;
  hipError_t ensure_side();
  struct LastRender {       // what read_stats needs of the last render
    std::vector<unsigned> rays, shadows;  // exhaustive pipeline: counts per generation (read back)
    unsigned last = 0, L = 0, n0 = 0, max_depth = 0;
    bool counted = false, exact_disc = false, bvh = false, fused = false;
    unsigned long long n_diag = 0, n_gen = 0, n_planes = 0, n_quads = 0;
    hipStream_t stream = nullptr;
  } lr_;
  // generation counts of the last render (fast path: from the host-mapped record; synchronises)
  hipError_t last_counts(std::vector<unsigned>& rays);
  bool last_bvh_ = false, last_fused_ = false;
  hipEvent_t gen_ev_ = nullptr;  // set_gen_event: recorded on the stream after generation gen_ev_g_'s launch
  int gen_ev_g_ = -1;
  bool gen_ev_done_ = false;
  unsigned blk_period_ = 0;  // the current render's block pattern (render())
  unsigned long long blk_mask_ = 0;
  bool profiling_ = false;
  int pmask_ = (1 << WF_NCLASS) - 1;
  std::vector<hipEvent_t> pev_;        // event pool (pairs)
  std::vector<int> pcls_;              // class of each recorded pair
  size_t pn_ = 0;                      // pairs recorded since profiling was enabled
  size_t pframes_ = 0;
  double prof_rays_[3] = {0, 0, 0};
  hipError_t pmark(hipStream_t s, int cls, bool begin);
};

}  // namespace rtamd
