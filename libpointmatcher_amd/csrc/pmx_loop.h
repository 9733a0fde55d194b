// pmx_loop.h — configuration and device state of the device-resident ICP
// loop (pmx_loop.hip, driven by pmx_loop_* in pmx_capi.hip).
#pragma once

#include "pmx_internal.h"

namespace pmx {

constexpr int kLoopHist = 64;      // Differential checker history ring (smoothLength < 64)
constexpr int kMaxCheckers = 8;
constexpr int kMaxLevels = 8;
// per-iteration diagnostics (pmx_loop_diag): a ring of kDiagCap records of
// kDiagWords 64-bit words, written by the step kernel at iteration % kDiagCap:
// [grid level of the match, quantile window (1 hit, 0 radix passes, -1 no
// window), pairs evaluated, full searches]
constexpr int kDiagCap = 1024;
constexpr int kDiagWords = 4;
// doubles of the iteration block the step reads (point-to-plane: <= 36 + 6 +
// 5 in the full layout; point-to-point: the second pass at 16..24)
constexpr int kStepRes = 48;

enum CheckKind { kCheckCounter = 0, kCheckDifferential = 1, kCheckBound = 2 };
// why the loop stopped
enum LoopReason { kLoopRunning = 0, kLoopCounter = 1, kLoopDifferential = 2, kLoopError = 3 };
// device-side error codes (mapped to pmx.h codes / messages by the host)
enum LoopErr {
    kLoopNoPoints = -1,   // PMX_E_NO_POINTS: "ErrorMnimizer: no point to minimize"
    kLoopNotRigid = -4,   // PMX_E_TRANSFORMATION
    kLoopRotNaN = -20,    // ConvergenceError("abs rotation norm not a number")
    kLoopTransNaN = -21,  // ConvergenceError("abs translation norm not a number")
    kLoopBound = -22,     // ConvergenceError("limit out of bounds ...")
};

struct Mat4d {
    double m[16];
};

struct LoopCfg {
    int rows;       // 3 (2-D) or 4 (3-D)
    int minimizer;  // 0 point-to-plane, 1 point-to-point
    int full;       // point-to-plane: the weighted reduction's layout (full A; a RobustOutlierFilter chain)
    int n_checkers;
    int checker_kind[kMaxCheckers];
    double checker_p[kMaxCheckers][3];
    // grid level adaptation (choose_level)
    int adaptive;
    int n_levels;       // levels built (the loop picks among them)
    int n_levels_all;   // levels of the grid (a coarser unbuilt one is requested: LoopState.want_level)
    double level_ppc[kMaxLevels];
    int64_t n_local;
    int reuse;  // the grid match's temporal reuse is on (level choice on full searches only)
    int knn;
    int tile_dispatch;  // both match forms enqueued; the step picks the next (pmx_step.h)
    int p2p_onepass;    // point-to-point: one moments pass (launch_p2point_moments layout), the step centres
};

template <typename T>
struct LoopState {
    T Titer[16];  // rows x rows
    int iter;     // iterations completed
    int done;
    int err;
    int reason;
    T cond[kMaxCheckers][2];     // checkers' condition variables
    T qhist[kLoopHist][4];       // Differential: quaternions (ring)
    T thist[kLoopHist][3];       //               translations
    int nhist;
    T bq0[4], bt0[3], brot2d0;   // Bound: initial rotation / translation
    double kept, nz, rejM, rejP, sw;  // last minimised iteration's ErrorElements statistics
    unsigned long long last_visited, touched;
    int last_level;
    int want_level;  // a coarser level the level rule wanted but was not built (the host builds it)
    int pad2[2];
    long long match_count;
    double level_cells[kMaxLevels];
    long long level_seen[kMaxLevels];
    T xsolve[6];  // the rank-deficient solve's result (loop_solve_rank_deficient)
};

template <typename T>
void launch_finalize_step(const double* partials, int nblocks, int nv, double* out, double* res, unsigned int* ticket,
                          LoopCtl* ctl, LoopState<T>* S, int* iter_err, unsigned long long* visited,
                          const T* means, const LoopCfg& cfg, T* trace, const int* spec_hit, long long* diag,
                          unsigned long long* vpart, hipStream_t s);
template <typename T>
void launch_loop_init(LoopCtl* ctl, LoopState<T>* S, const LoopCfg& cfg, const T* T0, int level, int prev_level,
                      const double* Tprev, int* iter_err, hipStream_t s);
template <typename T>
void launch_loop_step(LoopCtl* ctl, LoopState<T>* S, const double* res, const int* iter_err,
                      const unsigned long long* visited, const T* means, const LoopCfg& cfg, T* trace,
                      const int* spec_hit, long long* diag, hipStream_t s);

}  // namespace pmx
