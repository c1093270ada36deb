// tog_bwd_team.hpp — cost expansion + Riccati backward pass (std and square-root), column-per-lane.
//
// Reference: src/solvers/ilqr/backward_pass.jl:9-192 (+ cost expansion, ilqr_methods.jl:55-62,
// objective.jl:51-94, augmented_lagrangian_methods.jl:186-276).
//
// Mapping (MI355X, wave64): a TEAM of 16 lanes owns one trajectory, 4 trajectories per wave (8-lane
// teams, 8 per wave, for n <= 7). Lane c holds column c of every n x n / m x n block (S, A, Q.xx,
// Q.ux, K, ...) in registers and lane n holds the feed-forward column d. A product that needs another
// lane's column reads it from the team's LDS "bus" (column stores, broadcast reads — conflict-free),
// so every flop runs on registers. Householder QR is column-distributed: lane j forms reflector j and
// publishes it on the bus, lanes c > j apply it to their own column.
//
// Arithmetic contract: every output element is produced by one lane with the same
// fma sequence, in the same order, as oracle/tog_oracle.c (and the LDS kernel k_backward), so
// results are bit-identical. Terms that are exact zeros by structure (S below its diagonal, sparse
// constraint Jacobians) are skipped: fma(0, y, t) == t.
#pragma once
#include <type_traits>
// (included by tog_kernels.hpp after the LDS kernels; relies on their helpers)

namespace tog {

// Scheduling fence: keeps the compiler from hoisting a whole phase's bus reads (hundreds of LDS
// loads) ahead of their FMAs, which would need ~2x the registers of the logical working set.
#define TEAM_FENCE() asm volatile("" ::: "memory")

constexpr int PX = 20;  // rows with a state gradient per knot kept in registers (sqrt AL expansion)

template <class M>
struct TeamCfg {
  static constexpr int n = M::n, m = M::m, L = n + m;
  static constexpr int TEAM = (n + 1 <= 8) ? 8 : 16;
  static constexpr int TPW = WAVE / TEAM;
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  static constexpr int PU = 2 * m;  // rows with a control gradient per knot (bound constraints)
  // largest bus message: [A B] or W (n*L), S-update operands (3nm), tmp1 + s (32 + nm + n),
  // S / T (n*n + n), Quu (+B for :state), QR reflector (rows + 1)
  static constexpr int BUS =
      cmax(cmax(n * L, 3 * n * m), cmax(cmax(32 + n * m + n, n * n + n), cmax(m * m + n * m, n + PX + 2)));
  static constexpr int R2 = cmax(L * n, n * n + n);  // second region: W / S columns / T
  static constexpr int BUSP = cmax(BUS, n * L + R2);   // static part of the per-team stride (doubles)
  // sqrt: S [A B] goes to region 1 next to S B, so region 2 only holds the cond / chol_minus scratch
  static constexpr int R2S = cmax(3 * m * m, m * m + 1);
  static constexpr int BUSPS = cmax(BUS, n * L + R2S);
  static constexpr int RQ = cmax(2 * n, n + PX);  // register column of the Q.xx QR workspaces
};

struct RowInfo {  // one constraint row of the current knot (AL terms), 64 B
  double w, ws, g;
  double v[3];
  int idx[3];
  int nnz;
};
static_assert(sizeof(RowInfo) == 64, "RowInfo: 8 doubles of LDS (expand_team_stride)");

// Dynamic LDS layout of k_bwd_team (sizes from the host, bwd_team_stride / bwd_team_shmem):
//   per team (stride doubles): [S-region][region 1: n*L][region 2: R2 | R2S]
//   per block: int knot_cnt[N], int knot_nx[N] (dense-record test of the expansion records)
// S-region (persistent across knots, before region 1): S column-major and s (n*n + n); sqrt
// stores its upper factor dense, explicit zeros below the diagonal, so the rolled S [A B] product
// reads the oracle's dense operand without per-entry selects.
template <class M>
__host__ __device__ constexpr int sreg_size(bool) {  // S, s, then the knot's Q.uu (m*m)
  return M::n * M::n + M::n + M::m * M::m;
}
template <class M>
__host__ __device__ inline int bwd_team_stride(int /*pmax*/, int sqrt) {
  using C = TeamCfg<M>;
  int s = sqrt ? C::BUSPS : C::BUSP;
  s += sreg_size<M>(sqrt != 0);
  s += (34 - s % 32) % 32;  // s = 2 mod 32: the TPW teams' broadcast reads land on distinct banks
  return s;
}
inline size_t bwd_team_shmem(int stride, int tpw, int /*nrows*/, int N) {
  return sizeof(double) * (size_t)stride * tpw + sizeof(int) * 2 * (size_t)N;
}

// Expansion records (Bf.E, written by k_expand_team, read by k_bwd_team): per (trajectory, knot)
// a record of NE = n + m + m² + n² doubles
//   [0, n) Q.x | [n, n+m) Q.u | [n+m, n+m+m²) Q.uu | [n+m+m², NE) Q.xx   (column-major blocks;
// sqrt: Q.uu, Q.xx are the upper factors). Q.xx is written only at "dense" knots — the terminal
// knot and the knots whose AL terms change it (std: any row; sqrt: a row with a state gradient);
// elsewhere it is the problem constant (Q dt, or cholesky(Q dt).U), which the backward pass reads
// from DevProblem. Q.ux never depends on the trajectory for the team kernel's rows (bounds, goal,
// circles and spheres each have either a state or a control gradient): H dt (+ 0.0 where the std
// AL expansion adds its zero cu'Iμcx term, so the sign of a zero matches).
template <class M>
__host__ __device__ constexpr int ne_of() {
  return M::n + M::m + M::m * M::m + M::n * M::n;
}
constexpr int QPK = 4;  // packed-pattern rows per column the std expansion's row loop specialises for
template <bool SQRT, bool AL>
__device__ __forceinline__ bool knot_dense(int k, int N, int cnt, int nx) {
  return k == N - 1 || (AL && (SQRT ? nx > 0 : cnt > 0));
}
// LDS per team of k_expand_team (doubles): bus for the 8-lane QR, then RowInfo[pmax], xr/ur lists
// (pmax ints each), x[n], u[m]
template <class M>
__host__ __device__ inline int expand_team_stride(int pmax) {
  int s = 48 + pmax * 8 + pmax + M::n + M::m;
  return s + (s & 1);
}

// Host-side admissibility of the team kernel for a problem (otherwise the LDS kernel runs).
constexpr int TEAM_MAX_ROWS = 128;   // deduplicated row table cached in LDS
constexpr int TEAM_MAX_KNOTS = 1024;
inline bool team_rows_fit(const int* knot_off, const int* knot_cnt, const ConRow* rows, int N, int n, int m,
                          int nrows) {
  if (n + 1 > 16 || m > n || nrows > TEAM_MAX_ROWS || N > TEAM_MAX_KNOTS) return false;
  for (int k = 0; k < N; k++) {
    int nx = 0, nu = 0;
    if (knot_cnt[k] > PCAP) return false;
    for (int r = 0; r < knot_cnt[k]; r++) {
      const int t = rows[knot_off[k] + r].type;
      if (t == ROW_USER_INEQ || t == ROW_USER_EQ) return false;  // dense user rows: LDS kernel
      if (t == ROW_UMAX || t == ROW_UMIN) nu++;
      else nx++;
    }
    if (nx > PX || nu > 2 * m) return false;
  }
  return true;
}

// lane-parallel constraint evaluation into the team's row table (constraint_sets.jl:106-131,
// active_set augmented_lagrangian_methods.jl:190-195). cr: this knot's rows in the LDS row cache;
// x, u: the knot's state/control staged in LDS (u == nullptr at the terminal knot). The ordered
// lists of rows with a state / control gradient are built with ballots (team-uniform control flow).
template <class M>
__device__ __forceinline__ void team_rows(const DevBuffers& Bf, long long b, int k, int N, int pmax, int p,
                                          const ConRow* cr, const double* x, const double* u, RowInfo* rows,
                                          int* xr, int* ur, int& nx, int& nu, int team, int tl, int TEAM) {
  constexpr int n = M::n;
  const double* lam = Bf.lam + ((size_t)b * N + k) * pmax;
  const double* mu = Bf.mu + ((size_t)b * N + k) * pmax;
  const unsigned long long tmask = (TEAM >= 64 ? ~0ull : ((1ull << TEAM) - 1ull)) << (team * TEAM);
  const unsigned long long below = tmask & ((1ull << threadIdx.x) - 1ull);
  int cx = 0, cu = 0;
  for (int base = 0; base < p; base += TEAM) {
    const int r = base + tl;
    bool isx = false, isu = false;
    if (r < p) {
      const ConRow row = cr[r];
      const double c = row_value<false>(row, x, u);
      const double l = lam[r];
      const bool a = row_inequality<false>(row) ? ((c >= 0.0) || (l > 0.0)) : true;
      RowInfo ri;
      ri.w = a ? mu[r] : 0.0;
      ri.ws = a ? sqrt(mu[r]) : 0.0;
      ri.g = ri.w * c + l;
      ri.nnz = row_grad<false>(row, x, n, ri.idx, ri.v);
      rows[r] = ri;
      isu = (row.type == ROW_UMAX || row.type == ROW_UMIN);
      isx = !isu;
    }
    const unsigned long long bx = __ballot(isx) & tmask, bu = __ballot(isu) & tmask;
    if (isx) xr[cx + __popcll(bx & below)] = r;
    if (isu) ur[cu + __popcll(bu & below)] = r;
    cx += __popcll(bx);
    cu += __popcll(bu);
  }
  nx = cx;
  nu = cu;
}

// entry of a row's gradient at [x;u] index `col` (0 if structurally zero)
__device__ __forceinline__ double row_at(const RowInfo& r, int col) {
  double v = 0.0;
  for (int z = 0; z < r.nnz; z++)
    if (r.idx[z] == col) v = r.v[z];
  return v;
}

// Opaque copy (empty asm): addresses derived from it are recomputed where they are used instead of
// being hoisted out of the knot loop, kept live across it and spilled (a scratch reload waits on
// vmcnt, which also drains every global load in flight).
template <class T>
__device__ __forceinline__ T opaque(T v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Broadcast lane L's value to the 16 lanes of its DPP row (= its team when TEAM == 16): one 64-bit
// register move (v_mov_b64_dpp row_newbcast:L, gfx90a+ DPP64), no LDS round trip. All lanes of the
// team must be active (a disabled source lane is an invalid DPP source).
template <int L>
__device__ __forceinline__ double row_bcast(double v) {
  // (a frozen-poison `old` operand: every lane of the row has a valid source, so no copy of v is
  // needed to seed the destination)
  return __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(v), v, 0x150 + L, 0xF, 0xF, true);
}

// Broadcast lane L of each 4-lane group to the group (quad_perm [L,L,L,L], two 32-bit DPP moves)
template <int L>
__device__ __forceinline__ double quad_bcast(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(0), (int)(x & 0xffffffffll), L * 0x55,
                                             0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(0), (int)(x >> 32), L * 0x55, 0xF, 0xF,
                                             true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
// lane L of the team to the team: a 16-lane team is a DPP row, a 4-lane team a quad
template <int TW, int L>
__device__ __forceinline__ double team_bcast(double v) {
  static_assert(TW == 16 || TW == 4, "DPP team broadcasts: 16- or 4-lane teams");
  if constexpr (TW == 16) return row_bcast<L>(v);
  else return quad_bcast<L>(v);
}

// Lane i of each DPP row receives lane i-1's value, lane 0 of the row `old` (row_shr:1 with bound_ctrl
// off: the lane without a source keeps the old operand)
__device__ __forceinline__ double row_shr1_or(double v, double old) {
  const long long x = __builtin_bit_cast(long long, v), o = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffll), (int)(x & 0xffffffffll), 0x111, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(x >> 32), 0x111, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// Lane i of each DPP row receives lane i-1's value (row_shr:1, two 32-bit DPP moves: 64-bit DPP
// only has row_newbcast); lane 0 of the row receives 0.
__device__ __forceinline__ double row_shr1(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(0), (int)(x & 0xffffffffll), 0x111,
                                             0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(0), (int)(x >> 32), 0x111, 0xF, 0xF,
                                             true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// Column-distributed Householder QR (LAPACK dgeqr2/dlarfg as in Julia qr(P).R, and wqr): `a` is this
// lane's column (ROWS entries, the first `rows` in use — the rest are zero and inert) of a matrix
// whose columns live in lanes 0..COLS-1 of the team. When the first TOP rows form an upper-triangular
// block (the Cholesky factor being updated), rows j+1..TOP-1 of column j are exact zeros throughout
// the sweep (no reflector touches them), so they are skipped: their terms are fma(0, y, t) == t.
// FULL: rows == ROWS is known at compile time (no per-entry liveness selects).
struct QrNoPost {
  template <class J, class A>
  __device__ __forceinline__ void operator()(J, const A&) const {}
};
// POST (16-lane path): called after column step j as post(integral_constant j, a); row j of R is final
// then (no later reflector touches it), so a consumer may take R's rows as they are released.
template <int ROWS, int COLS, int TOP = 0, int TEAMW = 16, bool FULL = false, class POST = QrNoPost>
__device__ __forceinline__ void team_qr(double (&a)[ROWS], int rows, int tl, double* bus, const POST& post = POST{}) {
#define TQ_LIVE(i, j) ((FULL || TEAMW == 16 || TEAMW == 4 || (i) < rows) && !((i) > (j) && (i) < TOP))
  if constexpr (TEAMW == 16 || TEAMW == 4) {
    // Reflectors broadcast by DPP row_newbcast (the team is one DPP row; a 4-lane team: quad_perm). The lane-predicated parts
    // are written branch-free: every lane runs the reflector arithmetic on its own column (SIMT
    // issues it once either way) and lane j's results are selected once per step, and the update
    // uses w = 0 on lanes <= j, which leaves their live entries unchanged (x - 0, fma(v, 0, x)) and
    // only touches the dead reflector storage below their diagonals.
    // Contract v3 (oracle qr_R): the reflector stays unnormalised, v = [α-β; x], and
    // H y = y + v (v'y)/(β(α-β)). Per column j, lane j's pivot scalars and its column below the
    // diagonal reach the team by 64-bit DPP row broadcasts; lanes c > j then spend one fma per row
    // on v'y and one on the update. Rows past `rows` must be zero: they are inert (fma(0,0,s) == s,
    // fma(0,p,0) == 0), so the loops run over the compile-time ROWS with no per-row liveness tests.
    static_for<0, COLS>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      // lane tests recomputed per column from an opaque lane id: hoisted, the per-column exec masks
      // of every QR stay live across the knot loop as SGPR pairs and spill
      const int tq = opaque(tl);
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int i = j + 1; i < ROWS; i++)
        if (TQ_LIVE(i, j)) acc[(i - j - 1) & 3] = fma(a[i], a[i], acc[(i - j - 1) & 3]);
      const double ss = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      const double alpha = a[j];
      const double beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
      const double vd = alpha - beta;
      const double rd = (ss != 0.0) ? 1.0 / (beta * vd) : 0.0;  // 0: tau = 0, H = I
      if (tq == j && ss != 0.0) a[j] = beta;
      const double rdj = team_bcast<TEAMW, j>(rd), vdj = team_bcast<TEAMW, j>(vd);
      double v[ROWS];
#pragma unroll
      for (int i = j + 1; i < ROWS; i++)
        if (TQ_LIVE(i, j)) v[i] = team_bcast<TEAMW, j>(a[i]);
      if (tq > j && tq < COLS && rdj != 0.0) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = j + 1; i < ROWS; i++)
          if (TQ_LIVE(i, j)) a4[(i - j - 1) & 3] = fma(v[i], a[i], a4[(i - j - 1) & 3]);
        const double p = fma(vdj, a[j], (a4[0] + a4[1]) + (a4[2] + a4[3])) * rdj;
        a[j] = fma(vdj, p, a[j]);
#pragma unroll
        for (int i = j + 1; i < ROWS; i++)
          if (TQ_LIVE(i, j)) a[i] = fma(v[i], p, a[i]);
      }
      post(jc, a);
    });
    return;
  }
#pragma unroll
  for (int j = 0; j < COLS; j++) {
    if (j < rows) {
      double vd = 0.0;
      if (tl == j) {
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = j + 1; i < ROWS; i++)
          if (TQ_LIVE(i, j)) acc[(i - j - 1) & 3] = fma(a[i], a[i], acc[(i - j - 1) & 3]);
        const double ss = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        double rd = 0.0;  // contract v3 (see the 16-lane path): 0 means tau = 0, H = I
        if (ss != 0.0) {
          const double alpha = a[j];
          const double beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
          vd = alpha - beta;
          rd = 1.0 / (beta * vd);
#pragma unroll
          for (int i = j + 1; i < ROWS; i++)
            if (TQ_LIVE(i, j)) bus[i] = a[i];
          a[j] = beta;
        }
        bus[0] = rd;
      }
      vd = __shfl(vd, (int)(threadIdx.x - tl) + j, WAVE);  // lane j's α-β (every lane active here)
      team_sync();
      const double rd = bus[0];
      if (rd != 0.0 && tl > j && tl < COLS) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = j + 1; i < ROWS; i++)
          if (TQ_LIVE(i, j)) a4[(i - j - 1) & 3] = fma(bus[i], a[i], a4[(i - j - 1) & 3]);
        const double p = fma(vd, a[j], (a4[0] + a4[1]) + (a4[2] + a4[3])) * rd;
        a[j] = fma(vd, p, a[j]);
#pragma unroll
        for (int i = j + 1; i < ROWS; i++)
          if (TQ_LIVE(i, j)) a[i] = fma(bus[i], p, a[i]);
      }
      team_sync();
    }
  }
#undef TQ_LIVE
}

// cond(R) > thresh for an upper-triangular m x m R held by every lane of the team (backward_pass.jl:129;
// the oracle computes cond2 by one-sided Jacobi every time). The Frobenius bounds
// cond2 <= cF = |R|_F |R^-1|_F <= m cond2 decide almost every call; they are only bounds, so R^-1 is
// formed with the diagonal reciprocals rR (the gains solve reuses them) and the tests keep a 1e-12
// relative margin, far above the rounding of cF: a verdict taken here is the oracle's verdict. The
// Jacobi SVD of the ambiguous band runs on lane 0 of the team in LDS scratch `w` (m*m + 1 doubles)
// with the oracle's arithmetic, and its verdict is broadcast.
template <int m>
__device__ __forceinline__ bool cond_exceeds_team(const double (&R)[m][m], const double (&rR)[m], double thresh,
                                                  double* w, int tl) {
  double nr = 0.0, ni = 0.0;
#pragma unroll
  for (int c = 0; c < m; c++) {
    double ric[m];  // column c of R^-1 (zero below row c)
    ric[c] = rR[c];
#pragma unroll
    for (int j = c - 1; j >= 0; j--) {
      double t = 0.0;
#pragma unroll
      for (int l = j + 1; l <= c; l++) t = fma(R[j][l], ric[l], t);
      ric[j] = -t * rR[j];
    }
#pragma unroll
    for (int i = 0; i <= c; i++) {
      nr = fma(R[i][c], R[i][c], nr);
      ni = fma(ric[i], ric[i], ni);
    }
  }
  const double cF = sqrt(nr * ni);
  if (cF * (1.0 + 1e-12) <= thresh) return false;
  if (cF * (1.0 - 1e-12) > thresh * m) return true;
  // ambiguous band (team-uniform): one-sided Jacobi singular values on lane 0
  if (tl == 0) {
    double* A = w;
#pragma unroll
    for (int j = 0; j < m; j++)
#pragma unroll
      for (int i = 0; i < m; i++) A[i + m * j] = R[i][j];
    for (int sweep = 0; sweep < 60; sweep++) {
      double off = 0.0;
      for (int p = 0; p < m - 1; p++)
        for (int q = p + 1; q < m; q++) {
          double al = 0, be = 0, ga = 0;
          for (int i = 0; i < m; i++) {
            al += A[i + m * p] * A[i + m * p];
            be += A[i + m * q] * A[i + m * q];
            ga += A[i + m * p] * A[i + m * q];
          }
          if (ga == 0.0) continue;
          const double c0 = fabs(ga) / sqrt(al * be);
          off = fmax(off, c0);
          if (c0 < 1e-15) continue;
          const double zeta = (be - al) / (2.0 * ga);
          const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
          for (int i = 0; i < m; i++) {
            const double ap = A[i + m * p], aq = A[i + m * q];
            A[i + m * p] = cs * ap - sn * aq;
            A[i + m * q] = sn * ap + cs * aq;
          }
        }
      if (off < 1e-15) break;
    }
    double smax = 0.0, smin = INFINITY;
    for (int j = 0; j < m; j++) {
      double s2 = 0.0;
      for (int i = 0; i < m; i++) s2 += A[i + m * j] * A[i + m * j];
      smax = fmax(smax, sqrt(s2));
      smin = fmin(smin, sqrt(s2));
    }
    w[m * m] = ((smax / smin) > thresh) ? 1.0 : 0.0;
  }
  team_sync();
  const bool r = w[m * m] != 0.0;
  team_sync();
  return r;
}

// ============================================================================================
// k_expand_team: cost_expansion! (ilqr_methods.jl:55-62 -> objective.jl:51-94, cost.jl:183-198;
// AL terms augmented_lagrangian_methods.jl:186-276) for every (trajectory, knot) at once, into the
// expansion records Bf.E. The reference expands every knot before the backward pass starts, and
// nothing here depends on the cost-to-go, so this runs knot-parallel, off the Riccati recursion's
// serial chain: a TEAM-lane team per (trajectory, knot), consecutive knots of one trajectory in
// neighbouring teams (coalesced X, U, λ, μ reads and record writes). Lane c forms column c of Q.xx
// and Q.uu exactly as the fused expansion of round 2 did (same operations, same order: DESIGN.md §3).
// ============================================================================================
template <class M, bool SQRT, bool AL, bool TERM>
__device__ __forceinline__ void team_expand(const DevProblem* P, const DevBuffers& Bf, long long b, int k,
                                            double* tlds, int tl, int team) {
  using Cfg = TeamCfg<M>;
  constexpr int n = M::n, m = M::m, TEAM = Cfg::TEAM, RQ = Cfg::RQ, PU = Cfg::PU, NE = ne_of<M>();
  const int N = P->N, pmax = P->pmax;
  const double dt = P->dt;
  const bool colx = tl < n, colu = tl < m;
  const int c = colx ? tl : 0, cu = colu ? tl : 0;
  const double* xg = Bf.X + ((size_t)b * N + k) * n;
  const double* ug = TERM ? nullptr : Bf.U + ((size_t)b * (N - 1) + k) * m;
  double* bus = tlds;
  double Qxc[n], Quuc[m], Qu[m], Qxs;
  const double xc = xg[c];
  const int diag_mode = P->diag_cost;
  const CostView C_ = cost_at<n, m>(P, TERM ? 0 : k);  // stage knot k's cost (a time-varying Objective)
  if (!TERM && diag_mode == 2) {
    // diagonal cost with +0.0 off-diagonals (host-checked): the per-lane constants are one
    // diagonal entry each, the rest literal zeros -- the same values the general path loads
    const double Qcc = C_.Q[c + n * c], qc = C_.q[c];
    const double qd = SQRT ? C_.cQ[c + n * c] : Qcc * dt;
    const double rd = SQRT ? C_.cR[cu + m * cu] : C_.R[cu + m * cu] * dt;
    Qxs = ((fma(Qcc, xc, 0.0) + qc) + 0.0) * dt;
#pragma unroll
    for (int i = 0; i < m; i++) Qu[i] = ((fma(C_.R[i + m * i], ug[i], 0.0) + C_.r[i]) + 0.0) * dt;
#pragma unroll
    for (int i = 0; i < n; i++) Qxc[i] = (i == c) ? qd : 0.0;
#pragma unroll
    for (int i = 0; i < m; i++) Quuc[i] = (i == cu) ? rd : 0.0;
  } else if (!TERM) {
    double a = 0.0, bq = 0.0;
    if (diag_mode) {
      a = fma(C_.Q[c + n * c], xc, 0.0);
    } else {
#pragma unroll
      for (int j = 0; j < n; j++) a = fma(C_.Q[c + n * j], xg[j], a);
#pragma unroll
      for (int j = 0; j < m; j++) bq = fma(C_.H[j + m * c], ug[j], bq);
    }
    Qxs = ((a + C_.q[c]) + bq) * dt;
#pragma unroll
    for (int i = 0; i < m; i++) {
      double a2 = 0.0, b2 = 0.0;
      if (diag_mode) {
        a2 = fma(C_.R[i + m * i], ug[i], 0.0);
      } else {
#pragma unroll
        for (int j = 0; j < m; j++) a2 = fma(C_.R[i + m * j], ug[j], a2);
#pragma unroll
        for (int j = 0; j < n; j++) b2 = fma(C_.H[i + m * j], xg[j], b2);
      }
      Qu[i] = ((a2 + C_.r[i]) + b2) * dt;
    }
#pragma unroll
    for (int i = 0; i < n; i++) Qxc[i] = SQRT ? C_.cQ[i + n * c] : C_.Q[i + n * c] * dt;
#pragma unroll
    for (int i = 0; i < m; i++) Quuc[i] = SQRT ? C_.cR[i + m * cu] : C_.R[i + m * cu] * dt;
  } else {
    double a = 0.0;
    if (diag_mode) {
      a = fma(P->Qf[c + n * c], xc, 0.0);
    } else {
#pragma unroll
      for (int j = 0; j < n; j++) a = fma(P->Qf[c + n * j], xg[j], a);
    }
    Qxs = a + P->qf[c];
#pragma unroll
    for (int i = 0; i < n; i++) Qxc[i] = SQRT ? P->cQf[i + n * c] : P->Qf[i + n * c];
#pragma unroll
    for (int i = 0; i < m; i++) {
      Qu[i] = 0.0;
      Quuc[i] = 0.0;
    }
  }
  const int p = AL ? P->knot_cnt[k] : 0;
  if (AL && p > 0) {
    // rows area after the 8-lane QR bus
    RowInfo* rows = reinterpret_cast<RowInfo*>(tlds + 48);
    int* xr = reinterpret_cast<int*>(rows + pmax);
    int* ur = xr + pmax;
    double* xs = reinterpret_cast<double*>(ur + pmax);  // (2 pmax ints: 8-byte aligned)
    double* us = xs + n;
    if (colx) xs[tl] = xc;
    if (!TERM && colu) us[tl] = ug[tl];
    team_sync();
    int nx, nu;
    team_rows<M>(Bf, b, k, N, pmax, p, P->rows + P->knot_off[k], xs, TERM ? nullptr : us, rows, xr, ur, nx, nu,
                 team, tl, TEAM);
    team_sync();
    if (!SQRT && !TERM && P->qpat_on) {  // (qpat_on implies at most QPK pattern rows per column)
      // the same sums over the pattern (DevProblem::qpat): tX[i] can only change at column c's pattern rows,
      // so the row loop tests an entry's index against those (at most QPK) instead of all n; every (row,
      // entry) pair adds to the same sum in the same order, and the other tX[i] stay +0.0
      const unsigned int pc = colx ? as_const(P->qpat)[c] : 0u;
      int pidx[QPK];
      {
        unsigned int r_ = pc;
#pragma unroll
        for (int j = 0; j < QPK; j++) {
          pidx[j] = r_ ? __builtin_ctz(r_) : -1;
          r_ &= r_ - 1u;
        }
      }
      double tP[QPK], tUu[m];
#pragma unroll
      for (int j = 0; j < QPK; j++) tP[j] = 0.0;
#pragma unroll
      for (int i = 0; i < m; i++) tUu[i] = 0.0;
      for (int r = 0; r < p; r++) {
        const RowInfo& ri = rows[r];
        const double vxc = colx ? row_at(ri, c) : 0.0;
        const double vuc = colu ? row_at(ri, n + cu) : 0.0;
        if (vxc == 0.0 && vuc == 0.0) continue;
        for (int z = 0; z < ri.nnz; z++) {
          const int id = ri.idx[z];
          const double vw = ri.v[z] * ri.w;
#pragma unroll
          for (int j = 0; j < QPK; j++)
            if (id == pidx[j] && vxc != 0.0) tP[j] = fma(vw, vxc, tP[j]);
#pragma unroll
          for (int i = 0; i < m; i++)
            if (id == n + i && vuc != 0.0) tUu[i] = fma(vw, vuc, tUu[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < n; i++) {
        const int rk = __builtin_popcount(pc & ((1u << i) - 1u));
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < QPK; j++) t = (rk == j && (pc >> i & 1u)) ? tP[j] : t;
        Qxc[i] += t;
      }
#pragma unroll
      for (int i = 0; i < m; i++) Quuc[i] += tUu[i];
    } else if (!SQRT) {
      // Q.xx .+= cx'Iμ cx ; Q.uu .+= cu'Iμ cu ; Q.ux .+= cu'Iμ cx  (per-entry sums in row order; the
      // team kernel's rows never couple x and u, so the Q.ux term is an exact zero: ne_of)
      double tX[n], tUu[m];
#pragma unroll
      for (int i = 0; i < n; i++) tX[i] = 0.0;
#pragma unroll
      for (int i = 0; i < m; i++) tUu[i] = 0.0;
      for (int r = 0; r < p; r++) {
        const RowInfo& ri = rows[r];
        const double vxc = colx ? row_at(ri, c) : 0.0;
        const double vuc = (colu && !TERM) ? row_at(ri, n + cu) : 0.0;
        if (vxc == 0.0 && vuc == 0.0) continue;
        for (int z = 0; z < ri.nnz; z++) {
          const int id = ri.idx[z];
          const double vw = ri.v[z] * ri.w;
#pragma unroll
          for (int i = 0; i < n; i++)
            if (id == i && vxc != 0.0) tX[i] = fma(vw, vxc, tX[i]);
#pragma unroll
          for (int i = 0; i < m; i++)
            if (id == n + i && vuc != 0.0) tUu[i] = fma(vw, vuc, tUu[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < n; i++) Qxc[i] += tX[i];
      if (!TERM) {
#pragma unroll
        for (int i = 0; i < m; i++) Quuc[i] += tUu[i];
      }
    } else {
      // chol_plus!(Q.xx, Iμ_sqrt cx): QR of [Q.xx; ws.*cx]; rows without a state gradient are
      // zero rows of the stacked matrix and do not change R
      if (nx > 0) {
        double a[RQ];
#pragma unroll
        for (int i = 0; i < RQ; i++) {
          if (i < n) {
            a[i] = Qxc[i];
          } else if (i - n < nx) {
            const RowInfo& ri = rows[xr[i - n]];
            a[i] = ri.ws * row_at(ri, c);
          } else {
            a[i] = 0.0;
          }
        }
        team_qr<RQ, n, n, TEAM>(a, n + nx, tl, bus);
#pragma unroll
        for (int i = 0; i < n; i++) Qxc[i] = (i <= tl) ? a[i] : 0.0;
      }
      // chol_plus!(Q.uu, Iμ_sqrt cu)
      if (!TERM && nu > 0) {
        double a[m + PU];
#pragma unroll
        for (int i = 0; i < m + PU; i++) {
          if (i < m) {
            a[i] = Quuc[i];
          } else if (i - m < nu) {
            const RowInfo& ri = rows[ur[i - m]];
            // (control-bound rows: one gradient entry, ±1 at n + control)
            a[i] = ri.ws * ((ri.idx[0] == n + cu) ? ri.v[0] : 0.0);
          } else {
            a[i] = 0.0;
          }
        }
        // (16-lane teams run every QR over the zero-padded compile-time rows; 8-lane teams
        // specialise the common case, every control bounded on both sides)
        if (TEAM == 16 || nu == PU)
          team_qr<m + PU, m, m, TEAM, true>(a, m + PU, tl, bus);
        else
          team_qr<m + PU, m, m, TEAM>(a, m + nu, tl, bus);
#pragma unroll
        for (int i = 0; i < m; i++) Quuc[i] = (i <= tl) ? a[i] : 0.0;
      }
    }
    // Q.x .+= cx'g ; Q.u .+= cu'g
    {
      double tx = 0.0;
      for (int z = 0; z < nx; z++) {
        const RowInfo& ri = rows[xr[z]];
        const double v = colx ? row_at(ri, c) : 0.0;
        if (v != 0.0) tx = fma(v, ri.g, tx);
      }
      Qxs += tx;
      if (!TERM) {
        double tu[m];
#pragma unroll
        for (int i = 0; i < m; i++) tu[i] = 0.0;
        for (int z = 0; z < nu; z++) {
          const RowInfo& ri = rows[ur[z]];
          const int id = ri.idx[0];
#pragma unroll
          for (int i = 0; i < m; i++)
            if (id == n + i) tu[i] = fma(ri.v[0], ri.g, tu[i]);
        }
#pragma unroll
        for (int i = 0; i < m; i++) Qu[i] += tu[i];
      }
    }
  }
  // record (ne_of): Q.x, Q.u, Q.uu, and Q.xx at dense knots
  double* e = Bf.E + ((size_t)b * N + k) * NE;
  if (colx) e[tl] = Qxs;
  if (!TERM) {
    if (colu) {
      double qu = Qu[0];
#pragma unroll
      for (int i = 1; i < m; i++)
        if (tl == i) qu = Qu[i];
      e[n + tl] = qu;
#pragma unroll
      for (int i = 0; i < m; i++) e[n + m + i + m * tl] = Quuc[i];
    }
  }
  int nxk = 0;
  if (AL && SQRT) nxk = P->knot_nx[k];
  if (colx && knot_dense<SQRT, AL>(k, N, p, nxk)) {
#pragma unroll
    for (int i = 0; i < n; i++) e[n + m + m * m + i + n * tl] = Qxc[i];
  }
}

// mode 0: every knot; 1: only the dense ones (the others are on k_expand_u); 2: only the terminal knot
// (one team per trajectory: no stage knot is dense)
template <class M, int SQRTI, int ALI>
__global__ void __launch_bounds__(64) k_expand_team(const DevProblem* P, DevBuffers Bf, int mode) {
  using Cfg = TeamCfg<M>;
  extern __shared__ double expand_lds[];
  const int team = threadIdx.x / Cfg::TEAM, tl = threadIdx.x % Cfg::TEAM;
  const int N = P->N;
  const long long idx = (long long)blockIdx.x * Cfg::TPW + team;
  const long long slot = (mode == 2) ? idx : idx / N;
  const int k = (mode == 2) ? N - 1 : (int)(idx - slot * N);
  const long long b = traj_of_slot(Bf, slot, P->B);
  if (b < 0) return;  // whole teams return together (DPP broadcasts stay within a team)
  if (!Bf.st[b].active || Bf.st[b].ls_pend) return;
  if (mode == 1 && k < N - 1 && !(ALI && P->knot_nx[k] > 0)) return;
  double* tlds = expand_lds + (size_t)team * expand_team_stride<M>(P->pmax);
  if (k == N - 1)
    team_expand<M, SQRTI != 0, ALI != 0, true>(P, Bf, b, k, tlds, tl, team);
  else
    team_expand<M, SQRTI != 0, ALI != 0, false>(P, Bf, b, k, tlds, tl, team);
}

// k_expand_u: the square-root expansion of the knots whose Q.xx is the problem constant (stage knots
// without a state-gradient row: the record carries Q.x, Q.u and the Q.uu factor only) on 4-lane teams,
// 16 knots per wave. team_expand gives such a knot a 16-lane team of which only the m <= 4 Q.uu
// columns work; here lane c owns Q.uu's column c and Q.x's entries c, c + 4, ..., and every value is
// formed by team_expand's operations in its order (the Q.uu factor by the same column-distributed QR,
// its broadcasts within the quad). The dense knots (the terminal one, knots with state rows) stay on
// k_expand_team.
template <class M, bool AL>
__device__ __forceinline__ void quad_expand(const DevProblem* P, const DevBuffers& Bf, long long b, int k, int tl) {
  using Cfg = TeamCfg<M>;
  constexpr int n = M::n, m = M::m, PU = Cfg::PU, NE = ne_of<M>(), TQ = 4;
  static_assert(m <= TQ, "quad_expand: at most 4 controls");
  const int N = P->N, pmax = P->pmax;
  const double dt = P->dt;
  const bool colu = tl < m;
  const int cu = colu ? tl : 0;
  const double* xg = Bf.X + ((size_t)b * N + k) * n;
  const double* ug = Bf.U + ((size_t)b * (N - 1) + k) * m;
  constexpr int NXL = (n + TQ - 1) / TQ;  // Q.x entries of this lane: tl + TQ j
  double Qxs[NXL], Quuc[m], Qu[m];
  const int diag_mode = P->diag_cost;
  const CostView C_ = cost_at<n, m>(P, k);
  if (diag_mode == 2) {
#pragma unroll
    for (int j = 0; j < NXL; j++) {
      const int cc = tl + TQ * j < n ? tl + TQ * j : 0;
      Qxs[j] = ((fma(C_.Q[cc + n * cc], xg[cc], 0.0) + C_.q[cc]) + 0.0) * dt;
    }
#pragma unroll
    for (int i = 0; i < m; i++) Qu[i] = ((fma(C_.R[i + m * i], ug[i], 0.0) + C_.r[i]) + 0.0) * dt;
    const double rd = C_.cR[cu + m * cu];
#pragma unroll
    for (int i = 0; i < m; i++) Quuc[i] = (i == cu) ? rd : 0.0;
  } else {
#pragma unroll
    for (int j = 0; j < NXL; j++) {
      const int cc = tl + TQ * j < n ? tl + TQ * j : 0;
      double a = 0.0, bq = 0.0;
      if (diag_mode) {
        a = fma(C_.Q[cc + n * cc], xg[cc], 0.0);
      } else {
#pragma unroll
        for (int jj = 0; jj < n; jj++) a = fma(C_.Q[cc + n * jj], xg[jj], a);
#pragma unroll
        for (int jj = 0; jj < m; jj++) bq = fma(C_.H[jj + m * cc], ug[jj], bq);
      }
      Qxs[j] = ((a + C_.q[cc]) + bq) * dt;
    }
#pragma unroll
    for (int i = 0; i < m; i++) {
      double a2 = 0.0, b2 = 0.0;
      if (diag_mode) {
        a2 = fma(C_.R[i + m * i], ug[i], 0.0);
      } else {
#pragma unroll
        for (int j = 0; j < m; j++) a2 = fma(C_.R[i + m * j], ug[j], a2);
#pragma unroll
        for (int j = 0; j < n; j++) b2 = fma(C_.H[i + m * j], xg[j], b2);
      }
      Qu[i] = ((a2 + C_.r[i]) + b2) * dt;
    }
#pragma unroll
    for (int i = 0; i < m; i++) Quuc[i] = C_.cR[i + m * cu];
  }
  const int p = AL ? P->knot_cnt[k] : 0;
  if (AL && p > 0) {
    // The knot's rows, all control bounds (no state rows here, so team_rows' control-row list is the
    // row order itself and nu = p <= PU): row r on lane r % 4, evaluated as team_rows evaluates it, in
    // registers; lane c then takes row i's (√w, gradient entry, its index, g) from lane i % 4 by a quad
    // DPP broadcast. No LDS: the launch's occupancy is its register count's.
    constexpr int QR = (PU + TQ - 1) / TQ;
    const ConRow* cr = P->rows + P->knot_off[k];
    const double* lam = Bf.lam + ((size_t)b * N + k) * pmax;
    const double* mu = Bf.mu + ((size_t)b * N + k) * pmax;
    double rws[QR], rv[QR], rg[QR];
    int rid[QR];
#pragma unroll
    for (int q = 0; q < QR; q++) {
      const int r = tl + TQ * q;
      rws[q] = 0.0;
      rv[q] = 0.0;
      rg[q] = 0.0;
      rid[q] = -1;
      if (r < p) {
        const ConRow row = cr[r];
        const double c = row_value<false>(row, xg, ug);
        const double l = lam[r];
        const bool act = row_inequality<false>(row) ? ((c >= 0.0) || (l > 0.0)) : true;
        const double w = act ? mu[r] : 0.0;
        rws[q] = act ? sqrt(mu[r]) : 0.0;
        rg[q] = w * c + l;
        int gi[3];
        double gv[3];
        row_grad<false>(row, xg, n, gi, gv);
        rid[q] = gi[0];
        rv[q] = gv[0];
      }
    }
    const int nu = p;
    // row i's values on every lane of the quad (broadcast where used, so that no table stays live)
    auto idx_of = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      return __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(0), rid[i / TQ], (i % TQ) * 0x55, 0xF, 0xF,
                                         true);
    };
    // chol_plus!(Q.uu, Iμ_sqrt cu)
    {
      double a[m + PU];
#pragma unroll
      for (int i = 0; i < m; i++) a[i] = Quuc[i];
      static_for<0, PU>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const double ws = quad_bcast<i % TQ>(rws[i / TQ]), v = quad_bcast<i % TQ>(rv[i / TQ]);
        const int id = idx_of(ic);
        a[m + i] = (i < nu) ? ws * ((id == n + cu) ? v : 0.0) : 0.0;
      });
      team_qr<m + PU, m, m, TQ, true>(a, m + PU, tl, nullptr);
#pragma unroll
      for (int i = 0; i < m; i++) Quuc[i] = (i <= tl) ? a[i] : 0.0;
    }
    // Q.u .+= cu'g (Q.x .+= cx'g has no rows here)
    double tu[m];
#pragma unroll
    for (int i = 0; i < m; i++) tu[i] = 0.0;
    static_for<0, PU>([&](auto zc) {
      constexpr int z = decltype(zc)::value;
      const double v = quad_bcast<z % TQ>(rv[z / TQ]), g = quad_bcast<z % TQ>(rg[z / TQ]);
      const int id = idx_of(zc);
      if (z < nu) {
#pragma unroll
        for (int i = 0; i < m; i++)
          if (id == n + i) tu[i] = fma(v, g, tu[i]);
      }
    });
#pragma unroll
    for (int i = 0; i < m; i++) Qu[i] += tu[i];
    {  // Q.x .+= 0 (team_expand adds the empty sum: tx = 0.0)
#pragma unroll
      for (int j = 0; j < NXL; j++) Qxs[j] += 0.0;
    }
  }
  double* e = Bf.E + ((size_t)b * N + k) * NE;
#pragma unroll
  for (int j = 0; j < NXL; j++)
    if (tl + TQ * j < n) e[tl + TQ * j] = Qxs[j];
  if (colu) {
    double qu = Qu[0];
#pragma unroll
    for (int i = 1; i < m; i++)
      if (tl == i) qu = Qu[i];
    e[n + tl] = qu;
#pragma unroll
    for (int i = 0; i < m; i++) e[n + m + i + m * tl] = Quuc[i];
  }
}

template <class M, int ALI>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) k_expand_u(const DevProblem* P, DevBuffers Bf) {
  const int team = threadIdx.x / 4, tl = threadIdx.x % 4;
  const int N = P->N;
  const long long idx = (long long)blockIdx.x * 16 + team;
  const long long slot = idx / (N - 1);
  const int k = (int)(idx - slot * (N - 1));
  const long long b = traj_of_slot(Bf, slot, P->B);
  if (b < 0) return;  // whole teams return together (DPP broadcasts stay within a quad)
  if (!Bf.st[b].active || Bf.st[b].ls_pend) return;
  if (ALI && P->knot_nx[k] > 0) return;  // a dense knot: k_expand_team
  quad_expand<M, ALI != 0>(P, Bf, b, k, tl);
}

#ifndef TOG_BWD_WAVES
#define TOG_BWD_WAVES 2
#endif
#ifndef TOG_TAIL_PF
#define TOG_TAIL_PF 0  // measured slower (profiles/r3g_ab_tail.txt): the prefetch buffer's registers spill
#endif
#ifndef TOG_TAIL_TRI
#define TOG_TAIL_TRI 1
#endif
// (section timers: BPROF_DECL / BPROF / BPROF_FLUSH, defined in tog_kernels.hpp)
// WPE: waves per SIMD the register budget is sized for. The full batch runs WPE = TOG_BWD_WAVES (2:
// 256 registers, latency hidden by the second wave); the convergence tail -- few trajectories, most
// SIMDs idle -- runs WPE = 1 (512 registers, no spills on the serial chain; DevBuffers::tail).
template <class M, int SQRTI, int ALI, int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_bwd_team(const DevProblem* P, DevBuffers Bf, int flags) {
  // (P is deliberately not __restrict__: that would let LICM hoist ~100 loop-invariant problem
  // constants out of the knot loop and keep them in registers for the whole kernel)
  using Cfg = TeamCfg<M>;
  // ALI: bit 0 the AL expansion, bit 1 a time-varying Objective (TV: knot k's cost through cost_at, a table
  // every trajectory shares, so it stays in L2; a variant of its own so that the shared-cost kernels keep
  // their schedule)
  constexpr bool SQRT = SQRTI != 0, AL = (ALI & 1) != 0, TV = (ALI & 2) != 0;
  constexpr int n = M::n, m = M::m, L = n + m, TEAM = Cfg::TEAM, NQ = nq_of<M>(), NE = ne_of<M>();
  static_assert(m <= n && n + 1 <= TEAM, "team layout");
  extern __shared__ double team_lds[];
  const int team = threadIdx.x / TEAM, tl = threadIdx.x % TEAM;
  const long long bs = traj_of_slot(Bf, (long long)blockIdx.x * Cfg::TPW + team, P->B);
  const long long b = bs < 0 ? 0 : bs;
  const int N = P->N;
  const int stride = Bf.bwd_stride;
  constexpr int SREG = sreg_size<M>(SQRT);
  constexpr int SOFF = n * n;                            // offset of s in the S-region
  double* Sreg = team_lds + (size_t)team * stride;      // S (persistent between knots)
  double* QU = Sreg + SOFF + n;                          // Q.uu of the current knot (column-major)
  double* bus = Sreg + SREG;                             // region 1 | region 2
  // block-wide per-knot tables (dense-record test, knot_dense)
  int* kcnt = reinterpret_cast<int*>(team_lds + (size_t)Cfg::TPW * stride);
  int* knx = kcnt + N;
  if (AL) {
    for (int e = threadIdx.x; e < N; e += 64) {
      kcnt[e] = P->knot_cnt[e];
      knx[e] = P->knot_nx[e];
    }
    __syncthreads();
  }
  const bool live = bs >= 0 && Bf.st[b].active && !Bf.st[b].ls_pend;
  const bool store_S = (flags & TOG_BP_STORE_S) && Bf.Sdbg;
  const bool state_reg = (P->o.bp_reg_type == 1);
  const double dt = P->dt;
  const long long bb = live ? b : 0;  // safe base for idle teams (they never store)
  // per-trajectory bases, formed at each use from an opaque copy of bb (see opaque())
#define ABg (Bf.AB + (size_t)opaque(bb) * (N - 1) * n * L)
#define Kg (Bf.K + (size_t)opaque(bb) * (N - 1) * m * n)
#define dg (Bf.d + (size_t)opaque(bb) * (N - 1) * m)
#define Qs (Bf.Qscr + (size_t)opaque(bb) * N * NQ)
#define Eg (Bf.E + (size_t)opaque(bb) * N * NE)
  const bool colx = tl < n;  // this lane owns a state column
  const bool colu = tl < m;  // this lane owns a control column
  const int c = colx ? tl : 0;
  const int cu = colu ? tl : 0;
  // this lane's slot (base + tl * mul) of a team LDS array, formed at the use from an opaque copy of tl:
  // formed once, such addresses stay live across the knot loop and spill, and every spill reload waits
  // on vmcnt(0), which also drains the K/d stores and the loads in flight
  auto lane_at = [&](double* base, int mul) { return base + opaque(tl) * mul; };
  RegState s;
  s.rho = live ? Bf.st[b].rho : 0.0;
  s.drho = live ? Bf.st[b].drho : 0.0;
  s.flags = live ? Bf.st[b].flags : 0;
  const double rho0 = s.rho, drho0 = s.drho;
  bool faithful = false;  // replay mode reproducing the A.1 re-accumulation exactly
  int kmin = N - 1, restarts = 0;
  double dV0 = 0.0, dV1 = 0.0;
  double sown = 0.0;  // s[c] of the knot being produced
  bool done = !live;
  // PF (TOG_TAIL_PF, the 1-wave/SIMD tail variant): knot k-1's [A|B] columns and expansion record
  // loaded at the top of knot k. Off: measured 5 % slower at B = 1 (its buffer spills, and a spilled
  // reload waits on every load in flight), and the loads are only ~3 % of a knot.
  constexpr bool PF = (WPE == 1) && TOG_TAIL_PF;
  // TRI_SA: S [A B] over the upper factor's nonzero rows only, fully unrolled (the 2-wave/SIMD variant
  // keeps the rolled dense product: unrolled, its 256-register budget spills)
  constexpr bool TRI_SA = (WPE == 1) && TOG_TAIL_TRI;
  double pAc[n], pBc[n], pQxc[n], pQu[m], pQuuc[m], pQuxc[m], pQxs = 0.0;
  int pk = -1;  // knot whose inputs the p* registers hold
  BPROF_DECL

  // (the shared-cost variants read P's cost: every alternative form of this lambda measured -- a branch on the
  // per-knot table, strided cost pointers, packed Q.xx records read back here -- made the std AL backward
  // 20-30 % slower on config 4, profiles/r5s_*; so the per-knot cost is a template variant, TV)
  // Q blocks of knot k (terminal when TERM) from its expansion record (k_expand_team, ne_of):
  // this lane's columns of Q.xx, Q.uu, Q.ux, its Q.x entry and the whole Q.u
  auto expand = [&](const int k, auto term_c, double& Qxs, double(&Qu)[m], double(&Qxc)[n], double(&Quuc)[m],
                    double(&Quxc)[m]) {
    constexpr bool term = decltype(term_c)::value;
    const int tlk = opaque(tl);  // per-lane columns, formed per knot (not kept live across the loop)
    const int c = tlk < n ? tlk : 0, cu = tlk < m ? tlk : 0;
    const double* e = Eg + (size_t)k * NE;
    const int cnt = AL ? kcnt[k] : 0;
    Qxs = e[c];
    if (knot_dense<SQRT, AL>(k, N, cnt, AL ? knx[k] : 0)) {
#pragma unroll
      for (int i = 0; i < n; i++) Qxc[i] = e[n + m + m * m + i + n * c];
    } else if constexpr (TV) {
      const CostView C_ = cost_at<n, m>(P, k);
#pragma unroll
      for (int i = 0; i < n; i++) Qxc[i] = SQRT ? C_.cQ[i + n * c] : C_.Q[i + n * c] * dt;
    } else {
#pragma unroll
      for (int i = 0; i < n; i++) Qxc[i] = SQRT ? P->cQ[i + n * c] : P->Q[i + n * c] * dt;
    }
    if (!term) {
#pragma unroll
      for (int i = 0; i < m; i++) Qu[i] = e[n + i];
#pragma unroll
      for (int i = 0; i < m; i++) Quuc[i] = e[n + m + i + m * cu];
      const bool zterm = !SQRT && AL && cnt > 0;  // the std AL expansion's "+= cu'Iμcx" (an exact zero)
      const double* Hk = TV ? cost_at<n, m>(P, k).H : P->H;
#pragma unroll
      for (int i = 0; i < m; i++) {
        const double h = Hk[i + m * c] * dt;
        Quxc[i] = zterm ? h + 0.0 : h;
      }
    } else {
#pragma unroll
      for (int i = 0; i < m; i++) {
        Qu[i] = 0.0;
        Quuc[i] = 0.0;
        Quxc[i] = 0.0;
      }
    }
  };
  while (!done) {  // one attempt of the backward pass; a regularisation restart begins a new one
    TEAM_FENCE();
    {
      double Qxc[n], Quuc[m], Quxc[m], Qu[m], Qxs;
      expand(N - 1, std::integral_constant<bool, true>{}, Qxs, Qu, Qxc, Quuc, Quxc);
      // S[N] = Q[N] (backward_pass.jl:20-21 / :100-101)
      if (colx) {
#pragma unroll
        for (int i = 0; i < n; i++) {
          Sreg[i + n * tl] = (SQRT && i > tl) ? 0.0 : Qxc[i];
        }
        Sreg[SOFF + tl] = Qxs;
      }
      team_sync();
      if (store_S && colx) {
#pragma unroll
        for (int i = 0; i < n; i++) Bf.Sdbg[((size_t)b * N + (N - 1)) * n * n + i + n * tl] = Qxc[i];
        Bf.sdbg[((size_t)b * N + (N - 1)) * n + tl] = Qxs;
      }

    }
    dV0 = 0.0;
    dV1 = 0.0;
    bool restart = false;
    BPROF(0)  // terminal knot
    for (int k = N - 2; k >= 0; k--) {
      // keep the per-lane problem constants (cQ/cR/H/Q columns) loaded per knot: hoisted out of
      // the loop they would stay live across it and spill
      TEAM_FENCE();
      double Qxc[n], Quuc[m], Quxc[m], Qu[m], Qxs;
      double Ac[n], Bc[n];  // this lane's columns of ∇F[k] = [A|B]
      const bool replay = faithful && k >= kmin;
      const bool have_pf = PF && pk == k;  // knot k's inputs arrived during knot k+1 (neither its
                                           // [A|B] nor its expansion record changes between attempts)
      if (have_pf) {
#pragma unroll
        for (int i = 0; i < n; i++) {
          Ac[i] = pAc[i];
          Bc[i] = pBc[i];
          Qxc[i] = pQxc[i];
        }
#pragma unroll
        for (int i = 0; i < m; i++) {
          Qu[i] = pQu[i];
          Quuc[i] = pQuuc[i];
          Quxc[i] = pQuxc[i];
        }
        Qxs = pQxs;
      } else {
        const double* abk = ABg + (size_t)k * n * L;
#pragma unroll
        for (int i = 0; i < n; i++) {
          Ac[i] = abk[i + n * c];
          Bc[i] = abk[i + n * (n + cu)];
        }
      }
      if (PF && k > 0) {  // latency-sized variant: knot k-1's inputs load while knot k's chain runs
        const double* abk = ABg + (size_t)(k - 1) * n * L;
#pragma unroll
        for (int i = 0; i < n; i++) {
          pAc[i] = abk[i + n * c];
          pBc[i] = abk[i + n * (n + cu)];
        }
        expand(k - 1, std::integral_constant<bool, false>{}, pQxs, pQu, pQxc, pQuuc, pQuxc);
        pk = k - 1;
      }
      if (replay) {
        const double* q = Qs + (size_t)k * NQ;
        Qxs = q[c];
  #pragma unroll
        for (int i = 0; i < m; i++) Qu[i] = q[n + i];
  #pragma unroll
        for (int i = 0; i < n; i++) Qxc[i] = q[n + m + i + n * c];
  #pragma unroll
        for (int i = 0; i < m; i++) Quuc[i] = q[n + m + n * n + i + m * cu];
  #pragma unroll
        for (int i = 0; i < m; i++) Quxc[i] = q[n + m + n * n + m * m + i + m * c];
      } else if (!have_pf) {
        expand(k, std::integral_constant<bool, false>{}, Qxs, Qu, Qxc, Quuc, Quxc);
      }
    BPROF(1)  // expansion record loads
#ifdef TOG_BWD_PROF
    { volatile double sink_ = Ac[n - 1] + Bc[n - 1]; (void)sink_; }
#endif
    BPROF(17)  // [A B] loads
    // ---------------------------------------------------------------- Q.x += A's ; Q.u += B's
    {
      double t = 0.0;
#pragma unroll
      for (int l = 0; l < n; l++) t = fma(Ac[l], Sreg[SOFF + l], t);
      Qxs += t;
      double tu = 0.0;
#pragma unroll
      for (int l = 0; l < n; l++) tu = fma(Bc[l], Sreg[SOFF + l], tu);
      if constexpr (TEAM == 16) {
        static_for<0, m>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          Qu[i] += row_bcast<i>(tu);
        });
      } else {
        if (colu) bus[tl] = tu;
        team_sync();
#pragma unroll
        for (int i = 0; i < m; i++) Qu[i] += bus[i];
        team_sync();
      }
    }
    // [A B] columns on the bus (first region; the std path's products read them there)
    double* bus2 = bus + n * L;
    if (colx) {
#pragma unroll
      for (int i = 0; i < n; i++) bus[i + n * tl] = Ac[i];
    }
    if (colu) {
#pragma unroll
      for (int i = 0; i < n; i++) bus[i + n * (n + tl)] = Bc[i];
    }
    if (SQRT) team_sync();
    if (!SQRT) {
      // T1 = [A B]' S (L x n), then Q.xx += (A'S)A ; Q.uu += (B'S)B ; Q.ux += (B'S)A (backward_pass.jl:32-36)
      team_sync();
      // W = [A B]' S, column c per lane, written straight to the second bus region
      if (colx) {
        double Sc[n];
#pragma unroll
        for (int l = 0; l < n; l++) Sc[l] = Sreg[l + n * c];
#pragma unroll 1
        for (int i = 0; i < L; i++) {
          double t = 0.0;
#pragma unroll
          for (int l = 0; l < n; l++) t = fma(bus[l + n * i], Sc[l], t);
          bus2[i + L * tl] = t;
        }
      }
      team_sync();
      // reductions over l kept rolled (register accumulators, l ascending as in the oracle)
      double tq[n], tuu[m], tux[m];
#pragma unroll
      for (int i = 0; i < n; i++) tq[i] = 0.0;
#pragma unroll
      for (int i = 0; i < m; i++) {
        tuu[i] = 0.0;
        tux[i] = 0.0;
      }
#pragma unroll 1
      for (int l = 0; l < n; l++) {
        const double al = bus[l + n * c];
        const double bl = bus[l + n * (n + cu)];
#pragma unroll
        for (int i = 0; i < n; i++) tq[i] = fma(bus2[i + L * l], al, tq[i]);
#pragma unroll
        for (int i = 0; i < m; i++) {
          const double w = bus2[n + i + L * l];
          tuu[i] = fma(w, bl, tuu[i]);
          tux[i] = fma(w, al, tux[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < n; i++) Qxc[i] += tq[i];
#pragma unroll
      for (int i = 0; i < m; i++) {
        Quuc[i] += tuu[i];
        Quxc[i] += tux[i];
      }
      team_sync();
    } else {
      // tmp_x = S A, tmp_u = S B ; Q.ux += tmp_u' tmp_x ; Q.xx <- qr([Q.xx; tmp_x]).R ;
      // Q.uu <- qr([Q.uu; tmp_u]).R   (backward_pass.jl:112-118). Dense products, l ascending.
      double TX[n], TU[n];
#pragma unroll
      for (int i = 0; i < n; i++) {
        TX[i] = 0.0;
        TU[i] = 0.0;
      }
      // Column l of S is read from LDS in one burst (one wait per column). S is the upper factor: its
      // entries below the diagonal are exact +0.0, and the accumulators are never -0.0 (they start at
      // +0.0 and an fma whose exact result is zero rounds to +0.0), so the oracle's dense terms
      // fma(+0.0, a, t) == t for those rows are skipped (rows i <= l of column l only, ~half the work).
      if constexpr (TRI_SA) {
        static_for<0, n>([&](auto lc) {
          constexpr int l = decltype(lc)::value;
          double sl[l + 1];
          const double* Sl = Sreg + n * l;
#pragma unroll
          for (int i = 0; i <= l; i++) sl[i] = Sl[i];
          const double al = bus[l + n * c], bl = bus[l + n * (n + cu)];
          TEAM_FENCE();
#pragma unroll
          for (int i = 0; i <= l; i++) {
            TX[i] = fma(sl[i], al, TX[i]);
            TU[i] = fma(sl[i], bl, TU[i]);
          }
        });
      } else {
#pragma unroll 1
        for (int l = 0; l < n; l++) {
          double sl[n];
          const double* Sl = Sreg + n * l;
#pragma unroll
          for (int i = 0; i < n; i++) sl[i] = Sl[i];
          const double al = bus[l + n * c], bl = bus[l + n * (n + cu)];
          TEAM_FENCE();
#pragma unroll
          for (int i = 0; i < n; i++) {
            TX[i] = fma(sl[i], al, TX[i]);
            TU[i] = fma(sl[i], bl, TU[i]);
          }
        }
      }
      // Q.ux += tmp_u' tmp_x: tmp_u columns (lanes < m) then tmp_x columns go to region 1 ([A B]
      // is dead); per l one burst of reads, one wait. (A DPP form that skips the round trip makes the
      // compiler hoist the broadcasts and spill.)
      {
        team_sync();
        double* busx = bus + n * m;
        if (colu) {
#pragma unroll
          for (int i = 0; i < n; i++) bus[i + n * tl] = TU[i];
        }
        if (colx) {
#pragma unroll
          for (int i = 0; i < n; i++) busx[i + n * tl] = TX[i];
        }
        team_sync();
        double t[m];
#pragma unroll
        for (int i = 0; i < m; i++) t[i] = 0.0;
#pragma unroll 1
        for (int l = 0; l < n; l++) {
          double tu[m];
          const double tx = busx[l + n * c];
#pragma unroll
          for (int i = 0; i < m; i++) tu[i] = bus[l + n * i];
          TEAM_FENCE();
#pragma unroll
          for (int i = 0; i < m; i++) t[i] = fma(tu[i], tx, t[i]);
        }
#pragma unroll
        for (int i = 0; i < m; i++) Quxc[i] += t[i];
        team_sync();
      }
      BPROF(2)  // S [A B], Q.ux
      {
        double a[m + n];
#pragma unroll
        for (int i = 0; i < m + n; i++) a[i] = (i < m) ? Quuc[i] : TU[i - m];
        team_qr<m + n, m, m, TEAM>(a, m + n, tl, bus);
#pragma unroll
        for (int i = 0; i < m; i++) Quuc[i] = (i <= tl) ? a[i] : 0.0;
      }
      BPROF(3)  // QR Q.uu
      {
        double a[2 * n];
#pragma unroll
        for (int i = 0; i < 2 * n; i++) a[i] = (i < n) ? Qxc[i] : TX[i - n];
        team_qr<2 * n, n, n, TEAM>(a, 2 * n, tl, bus);
#pragma unroll
        for (int i = 0; i < n; i++) Qxc[i] = (i <= tl) ? a[i] : 0.0;
      }
      BPROF(4)  // QR Q.xx
    }
    if (faithful) {
      double* q = Qs + (size_t)k * NQ;
      if (colx) {
        q[tl] = Qxs;
#pragma unroll
        for (int i = 0; i < n; i++) q[n + m + i + n * tl] = Qxc[i];
#pragma unroll
        for (int i = 0; i < m; i++) q[n + m + n * n + m * m + i + m * tl] = Quxc[i];
      }
      if (colu) {
#pragma unroll
        for (int i = 0; i < m; i++) q[n + m + n * n + i + m * tl] = Quuc[i];
      }
      if (tl == 0) {
#pragma unroll
        for (int i = 0; i < m; i++) q[n + i] = Qu[i];
      }
      kmin = k < kmin ? k : kmin;
    }
    // ---------------------------------------------------------------- regularise, test, gains
    // (backward_pass.jl:38-48 / :120-126). Every lane needs the full Q.uu: all-gather its columns.
    if (colu) {
      double* qc = lane_at(QU, m);
#pragma unroll
      for (int i = 0; i < m; i++) qc[i] = Quuc[i];
      if (state_reg) {  // (:state regularisation only; reloaded to keep [A|B] out of registers)
        const double* bk = ABg + (size_t)k * n * L + n * (n + tl);
#pragma unroll
        for (int i = 0; i < n; i++) bus[m * m + i + n * tl] = bk[i];
      }
    }
    team_sync();
    // right-hand side of this lane: Qux_reg column (state reg adds ρ B'A), or Q.u for lane n
    double col[m];
    if (colx) {
#pragma unroll
      for (int i = 0; i < m; i++) col[i] = Quxc[i];
      if (state_reg) {
        const double* ak = ABg + (size_t)k * n * L + n * c;
        double t[m];
#pragma unroll
        for (int i = 0; i < m; i++) t[i] = 0.0;
#pragma unroll 1
        for (int l = 0; l < n; l++) {
          const double a = ak[l];
#pragma unroll
          for (int i = 0; i < m; i++) t[i] = fma(bus[m * m + l + n * i], a, t[i]);
        }
#pragma unroll
        for (int i = 0; i < m; i++) col[i] += s.rho * t[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < m; i++) col[i] = Qu[i];
    }
    double F[m][m], rF[m];
    bool ok = true;
    int piv[m];
    if (!SQRT) {
#pragma unroll
      for (int j = 0; j < m; j++)
#pragma unroll
        for (int i = 0; i < m; i++) F[i][j] = QU[i + m * j];
      if (!state_reg) {
#pragma unroll
        for (int i = 0; i < m; i++) F[i][i] += s.rho;
      } else {
        double t[m][m];
#pragma unroll
        for (int j = 0; j < m; j++)
#pragma unroll
          for (int i = 0; i < m; i++) t[i][j] = 0.0;
#pragma unroll 1
        for (int l = 0; l < n; l++) {
          double bl[m];
#pragma unroll
          for (int i = 0; i < m; i++) bl[i] = bus[m * m + l + n * i];
#pragma unroll
          for (int j = 0; j < m; j++)
#pragma unroll
            for (int i = 0; i < m; i++) t[i][j] = fma(bl[i], bl[j], t[i][j]);
        }
#pragma unroll
        for (int j = 0; j < m; j++)
#pragma unroll
          for (int i = 0; i < m; i++) F[i][j] += s.rho * t[i][j];
      }
      team_sync();
      // isposdef(Hermitian(Quu_reg)): Cholesky of the upper triangle
      {
        double U[m][m];
#pragma unroll
        for (int j = 0; j < m; j++) {
          double d0 = F[j][j];
#pragma unroll
          for (int l = 0; l < j; l++) d0 -= U[l][j] * U[l][j];
          if (!(d0 > 0.0)) ok = false;
          const double ujj = sqrt(d0);
          U[j][j] = ujj;
#pragma unroll
          for (int cc = j + 1; cc < m; cc++) {
            double t = F[j][cc];
#pragma unroll
            for (int l = 0; l < j; l++) t -= U[l][j] * U[l][cc];
            U[j][cc] = t / ujj;
          }
        }
      }
      // LU with partial pivoting (dgetrf; Julia `\`)
#pragma unroll
      for (int kk = 0; kk < m; kk++) {
        int p = kk;
        double amax = fabs(F[kk][kk]);
#pragma unroll
        for (int i = kk + 1; i < m; i++)
          if (fabs(F[i][kk]) > amax) {
            amax = fabs(F[i][kk]);
            p = i;
          }
        piv[kk] = p;
#pragma unroll
        for (int i = kk + 1; i < m; i++)
          if (i == p) {
#pragma unroll
            for (int j = 0; j < m; j++) {
              const double t = F[kk][j];
              F[kk][j] = F[i][j];
              F[i][j] = t;
            }
          }
        const double akk = F[kk][kk];
        if (akk != 0.0) {
          const double r = 1.0 / akk;
#pragma unroll
          for (int i = kk + 1; i < m; i++) F[i][kk] *= r;
        }
#pragma unroll
        for (int j = kk + 1; j < m; j++)
#pragma unroll
          for (int i = kk + 1; i < m; i++) F[i][j] = fma(-F[i][kk], F[kk][j], F[i][j]);
      }
    } else {
      team_sync();
      // Quu_reg = qr([Q.uu; sqrt(ρ) I]).R (:control) or qr([Q.uu; sqrt(ρ) B]).R (:state),
      // column-distributed over lanes < m, then all-gathered
      {
        const double sr = sqrt(s.rho);
        // one instantiation per regularisation type (uniform branch), each with its exact row count
        auto qr_reg = [&](auto& a) {
          constexpr int RR = sizeof(a) / sizeof(a[0]);
#pragma unroll
          for (int i = 0; i < RR; i++) {
            double v = 0.0;
            if (i < m) v = Quuc[i];
            else if (state_reg) v = sr * ABg[(size_t)k * n * L + n * (n + cu) + (i - m)];
            else if (i - m == tl) v = sr;
            a[i] = v;
          }
          team_qr<RR, m, m, TEAM, true>(a, RR, tl, bus);
          if constexpr (TEAM == 16) {
            static_for<0, m>([&](auto jc) {
              constexpr int j = decltype(jc)::value;
#pragma unroll
              for (int i = 0; i < m; i++) F[i][j] = (i <= j) ? row_bcast<j>(a[i]) : 0.0;
            });
          } else {
            if (colu) {
#pragma unroll
              for (int i = 0; i < m; i++) bus[i + m * tl] = (i <= tl) ? a[i] : 0.0;
            }
          }
        };
        if (state_reg) {
          double a[m + n];
          qr_reg(a);
        } else {
          double a[2 * m];
          qr_reg(a);
        }
      }
      if constexpr (TEAM != 16) {
        team_sync();
#pragma unroll
        for (int j = 0; j < m; j++)
#pragma unroll
          for (int i = 0; i < m; i++) F[i][j] = bus[i + m * j];
        team_sync();
      }
#pragma unroll
      for (int j = 0; j < m; j++) rF[j] = 1.0 / F[j][j];
      ok = !cond_exceeds_team<m>(F, rF, 1e8, bus2, tl);
    }
    BPROF(5)  // regularise + cond
    if (!ok) {
      // non-PD / cond > 1e8: increase ρ and restart at N-1; Q blocks are NOT re-expanded (A.1)
      if (!faithful) {
        faithful = true;  // replay this call from its start in faithful mode
        s.rho = rho0;
        s.drho = drho0;
        restarts = 0;
        kmin = N - 1;
      } else {
        reg_increase(P, s);
        restarts++;
        if (restarts > TOG_BP_MAX_RESTARTS) {  // restart cap (tog.h): the trajectory stops
          s.flags |= TOG_TRAJ_MAX_REG | TOG_TRAJ_BP_ABORTED;
          done = true;
        }
      }
      restart = true;
      break;
    }
    if (!SQRT) {
      // K = -(Quu_reg \ Qux_reg), d = -(Quu_reg \ Q.u)
#pragma unroll
      for (int kk = 0; kk < m; kk++) {
#pragma unroll
        for (int i = kk + 1; i < m; i++)
          if (i == piv[kk]) {
            const double t = col[kk];
            col[kk] = col[i];
            col[i] = t;
          }
      }
#pragma unroll
      for (int j = 0; j < m; j++)
#pragma unroll
        for (int i = j + 1; i < m; i++) col[i] = fma(-F[i][j], col[j], col[i]);
#pragma unroll
      for (int j = m - 1; j >= 0; j--) {
        col[j] /= F[j][j];
#pragma unroll
        for (int i = 0; i < j; i++) col[i] = fma(-F[i][j], col[j], col[i]);
      }
    } else {
      // K = -Quu_reg \ (Quu_reg' \ Qux_reg); contract v2: multiply by the diagonal reciprocals
      // (rF: the diagonal reciprocals formed for the cond test)
#pragma unroll
      for (int j = 0; j < m; j++) {
        const double xj = col[j] * rF[j];
        col[j] = xj;
#pragma unroll
        for (int i = j + 1; i < m; i++) col[i] = fma(-F[j][i], xj, col[i]);
      }
#pragma unroll
      for (int j = m - 1; j >= 0; j--) {
        const double xj = col[j] * rF[j];
        col[j] = xj;
#pragma unroll
        for (int i = j - 1; i >= 0; i--) col[i] = fma(-F[i][j], xj, col[i]);
      }
    }
    BPROF(6)  // gains solve
    double Kc[m];
#pragma unroll
    for (int i = 0; i < m; i++) Kc[i] = -1.0 * col[i];
    double d[m];
    if constexpr (TEAM == 16) {
#pragma unroll
      for (int i = 0; i < m; i++) d[i] = row_bcast<n>(Kc[i]);
    } else {
      if (tl == n) {
#pragma unroll
        for (int i = 0; i < m; i++) bus[i] = Kc[i];
      }
      team_sync();
#pragma unroll
      for (int i = 0; i < m; i++) d[i] = bus[i];
      team_sync();
    }
    if (colx) {
#pragma unroll
      for (int i = 0; i < m; i++) Kg[(size_t)k * m * n + i + m * tl] = Kc[i];
    }
    if (tl == n) {
#pragma unroll
      for (int i = 0; i < m; i++) dg[(size_t)k * m + i] = Kc[i];
    }
    if (!SQRT) {
      double KtQ[m];  // row c of K' Q.uu
#pragma unroll
      for (int j = 0; j < m; j++) {
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) t = fma(Kc[l], QU[l + m * j], t);
        KtQ[j] = t;
      }
      // s[c] = Q.x[c] + (K'Q.uu)[c,:] d + K[:,c]'Q.u + Q.ux[:,c]'d
      {
        double a = 0.0, b2 = 0.0, c2 = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) {
          a = fma(KtQ[l], d[l], a);
          b2 = fma(Kc[l], Qu[l], b2);
          c2 = fma(Quxc[l], d[l], c2);
        }
        sown = ((Qxs + a) + b2) + c2;
      }
      // T[i][c] = Q.xx[i][c] + (K'Q.uu)[i,:]K[:,c] + K[:,i]'Q.ux[:,c] + Q.ux[:,i]'K[:,c]
      if (colx) {
#pragma unroll
        for (int l = 0; l < m; l++) {
          bus[l + m * tl] = KtQ[l];
          bus[n * m + l + m * tl] = Kc[l];
          bus[2 * n * m + l + m * tl] = Quxc[l];
        }
      }
      team_sync();
      double T[n];
      {
        double ta[n], tb[n], tc[n];
#pragma unroll
        for (int i = 0; i < n; i++) {
          ta[i] = 0.0;
          tb[i] = 0.0;
          tc[i] = 0.0;
        }
#pragma unroll 1
        for (int l = 0; l < m; l++) {
          const double kl = bus[n * m + l + m * c];       // K[l][c]
          const double ql = bus[2 * n * m + l + m * c];   // Q.ux[l][c]
#pragma unroll
          for (int i = 0; i < n; i++) {
            ta[i] = fma(bus[l + m * i], kl, ta[i]);
            tb[i] = fma(bus[n * m + l + m * i], ql, tb[i]);
            tc[i] = fma(bus[2 * n * m + l + m * i], kl, tc[i]);
          }
        }
#pragma unroll
        for (int i = 0; i < n; i++) T[i] = ((Qxc[i] + ta[i]) + tb[i]) + tc[i];
      }
      team_sync();
      // S = 0.5 (T + T'); all-gather s
      if (colx) {
#pragma unroll
        for (int i = 0; i < n; i++) bus[i + n * tl] = T[i];
      }
      team_sync();
      if (colx) {
#pragma unroll
        for (int i = 0; i < n; i++) Sreg[i + n * tl] = 0.5 * (T[i] + bus[c + n * i]);
        Sreg[SOFF + tl] = sown;
      }
      team_sync();
      {
        double a = 0.0, b2 = 0.0;
#pragma unroll
        for (int i = 0; i < m; i++) a = fma(d[i], Qu[i], a);
#pragma unroll
        for (int j = 0; j < m; j++) {
          double t = 0.0;
#pragma unroll
          for (int i = 0; i < m; i++) t = fma(0.5 * d[i], QU[i + m * j], t);
          b2 = fma(t, d[j], b2);
        }
        dV0 += a;
        dV1 += b2;
      }
    } else {
      double Ud[m], KtU[m];  // Q.uu d ; row c of K' Q.uu'
#pragma unroll
      for (int i = 0; i < m; i++) {
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) t = fma(QU[i + m * l], d[l], t);
        Ud[i] = t;
      }
#pragma unroll
      for (int j = 0; j < m; j++) {
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) t = fma(Kc[l], QU[j + m * l], t);
        KtU[j] = t;
      }
      {
        double a = 0.0, b2 = 0.0, c2 = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) {
          a = fma(KtU[l], Ud[l], a);
          b2 = fma(Kc[l], Qu[l], b2);
          c2 = fma(Quxc[l], d[l], c2);
        }
        sown = ((Qxs + a) + b2) + c2;
      }
      // tmp1 = (Q.xx') \ Q.ux' by distributed forward substitution: lane i owns row i of tmp1
      double t1[m];
#pragma unroll
      for (int i = 0; i < m; i++) t1[i] = Quxc[i];
      // contract v2: x_j = b_j·(1/U_jj); lane j forms the reciprocal of its diagonal entry up front
      double dgx = Qxc[0];
#pragma unroll
      for (int j = 1; j < n; j++)
        if (tl == j) dgx = Qxc[j];
      const double rdiag = 1.0 / dgx;
      if constexpr (TEAM == 16) {
        static_for<0, n>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if (tl == j) {
#pragma unroll
            for (int i = 0; i < m; i++) t1[i] = t1[i] * rdiag;
          }
          double xj[m];
#pragma unroll
          for (int i = 0; i < m; i++) xj[i] = row_bcast<j>(t1[i]);
          if (tl > j && colx) {
#pragma unroll
            for (int i = 0; i < m; i++) t1[i] = fma(-Qxc[j], xj[i], t1[i]);
          }
        });
      } else {
#pragma unroll
        for (int j = 0; j < n; j++) {
          if (tl == j) {
#pragma unroll
            for (int i = 0; i < m; i++) {
              t1[i] = t1[i] * rdiag;
              bus[i] = t1[i];
            }
          }
          team_sync();
          if (tl > j && colx) {
#pragma unroll
            for (int i = 0; i < m; i++) t1[i] = fma(-Qxc[j], bus[i], t1[i]);
          }
          team_sync();
        }
      }
      BPROF(7)  // K/d store, s, tmp1
      // all-gather tmp1 (row-major at bus[TB + r*m + j]) and s
      constexpr int TB = 32;
      if (colx) {
        double* tr = lane_at(bus + TB, m);
#pragma unroll
        for (int i = 0; i < m; i++) tr[i] = t1[i];
      }
      team_sync();
      // tmp2 = chol_minus(Q.uu, tmp1): lowrankdowndate! by each row of tmp1 (backward_pass.jl:186-192).
      // Systolic schedule: lane i owns row i of the factor; the downdate of (row r, column i) needs
      // only (r, i-1) and (r-1, i), so step t runs (r = t - i, i) on every lane i < m: n+m-1 steps
      // instead of n*m, each (r, i) with exactly the oracle's operations. Lane i keeps its row and
      // the travelling x in a frame shifted by i (u[k] = R[i][i+k], w[k] = x[i+k]; slots k >= m-i
      // carry don't-care values), so the pivot is always u[0], w[0] with no per-lane selects, and
      // lane i-1 hands lane i its w[1..] (DPP row_shr:1 on 16-lane teams).
      const double* U2p;  // tmp2 (column-major): the downdated factor
      bool pd_abort = false;
      {
        double u[m], w[m], wn[m];
        const double* qd = lane_at(QU, m + 1);  // (Q.uu's diagonal entry of row tl)
#pragma unroll
        for (int k = 0; k < m; k++) {
          u[k] = (colu && tl + k < m) ? qd[m * k] : 0.0;
          w[k] = 0.0;
          wn[k] = bus[TB + k];  // lane 0: row 0 of tmp1 (the other lanes ignore wn)
        }
        // contract v4 (oracle chol_minus): s = x_i·(1/R_ii) with the diagonal reciprocal carried by
        // products (1/(c R_ii) = (1/R_ii)(1/c)), 1/c = tog_rsqrt(1 - s²), c = (1 - s²)(1/c)
        double ru = 1.0 / u[0];
        bool okd = true;
        if constexpr (TEAM == 16) {
          // Branch-free steps: every lane runs the rotation each step and keeps its row only while it
          // holds an active (row r, column i) pair. Lane 0 takes row t of tmp1 from the bus (read a
          // step ahead, the same address on every lane), the others lane i-1's x (DPP row_shr:1).
          // A lane's travelling x is read by lane i+1 only on the step after one it was active on.
#pragma unroll 1
          for (int t = 0; t < n + m - 1; t++) {
            const int r = t - tl;
            const bool act = colu && r >= 0 && r < n;
            double x[m];
#pragma unroll
            for (int k = 0; k + 1 < m; k++) x[k] = row_shr1(w[k + 1]);  // lane i-1's x from step t-1
            x[m - 1] = 0.0;
#pragma unroll
            for (int k = 0; k < m; k++) x[k] = (tl == 0) ? wn[k] : x[k];
            const int rn = t + 1 < n ? t + 1 : n - 1;  // lane 0's next row of tmp1
#pragma unroll
            for (int k = 0; k < m; k++) wn[k] = bus[TB + rn * m + k];
            const double sn = x[0] * ru;
            const double s2 = sn * sn;
            okd = okd && !(act && s2 > 1.0);
            const double y = 1.0 - s2;
            const double rc = tog_rsqrt(y);
            const double cs = tog_rs_c(y, rc);
            w[0] = x[0];
#pragma unroll
            for (int k = 1; k < m; k++) {
              const double tmp = (u[k] - sn * x[k]) * rc;
              w[k] = cs * x[k] - sn * tmp;
              u[k] = act ? tmp : u[k];
            }
            u[0] = act ? cs * u[0] : u[0];
            ru = act ? ru * rc : ru;
          }
        } else {
          double* msg = bus2;  // [2][m][m]: lane i-1 -> lane i messages (8-lane teams)
#pragma unroll 1
          for (int t = 0; t < n + m - 1; t++) {
            const int r = t - tl;
            if (colu && r >= 0 && r < n) {
              if (tl == 0) {
#pragma unroll
                for (int k = 0; k < m; k++) w[k] = wn[k];
                const int rn = r + 1 < n ? r + 1 : r;  // prefetch the next row of tmp1
#pragma unroll
                for (int k = 0; k < m; k++) wn[k] = bus[TB + rn * m + k];
              } else {
                const double* in = msg + ((t - 1) & 1) * m * m + (tl - 1) * m;
#pragma unroll
                for (int k = 0; k + 1 < m; k++) w[k] = in[k + 1];
              }
              const double sn = w[0] * ru;
              const double s2 = sn * sn;
              if (s2 > 1.0) okd = false;
              const double y = 1.0 - s2;
              const double rc = tog_rsqrt(y);
              const double cs = tog_rs_c(y, rc);
              u[0] = cs * u[0];
              ru = ru * rc;
#pragma unroll
              for (int k = 1; k < m; k++) {
                const double tmp = (u[k] - sn * w[k]) * rc;
                w[k] = cs * w[k] - sn * tmp;
                u[k] = tmp;
              }
              double* out = msg + (t & 1) * m * m + tl * m;
#pragma unroll
              for (int k = 0; k < m; k++) out[k] = w[k];
            }
            team_sync();
          }
        }
        const unsigned long long tmask = (TEAM >= 64 ? ~0ull : ((1ull << TEAM) - 1ull)) << (team * TEAM);
        const bool fail = (__ballot(!okd) & tmask) != 0ull;
        if (colu) {
          // row tl of tmp2 (column-major): entry (tl, jj) is u[jj - tl] from the diagonal on, 0 below it;
          // written branch-free, every column of the row
          double* tr = lane_at(bus2 + 2 * m * m, 1);
          const int tq = opaque(tl);
          static_for<0, m>([&](auto jc) {
            constexpr int jj = decltype(jc)::value;
            double v = 0.0;
            static_for<0, jj + 1>([&](auto kc) {
              constexpr int k = decltype(kc)::value;
              v = (tq + k == jj) ? u[k] : v;
            });
            tr[m * jj] = v;
          });
        }
        team_sync();
        U2p = bus2 + 2 * m * m;
        pd_abort = fail;
      }
      BPROF(8)  // chol_minus
      if (pd_abort) {  // lowrankdowndate! throws PosDefException: this trajectory's solve stops
        s.flags |= TOG_TRAJ_SQRT_PD_FAIL | TOG_TRAJ_BP_ABORTED;
        done = true;
        restart = true;
        break;
      }
      // S[k] = qr([Q.xx + tmp1 K; tmp2 K]).R
      {
        constexpr int RS = n + m;
        double a[RS];
        {
          double v[n];
#pragma unroll
          for (int i = 0; i < n; i++) v[i] = 0.0;
#pragma unroll
          for (int l = 0; l < m; l++) {
#pragma unroll
            for (int i = 0; i < n; i++) v[i] = fma(bus[TB + i * m + l], Kc[l], v[i]);
            TEAM_FENCE();
          }
#pragma unroll
          for (int i = 0; i < n; i++) a[i] = Qxc[i] + v[i];
        }
#pragma unroll
        for (int i = 0; i < m; i++) {
          double v = 0.0;
#pragma unroll
          for (int l = 0; l < m; l++) v = fma(U2p[i + m * l], Kc[l], v);
          a[n + i] = v;
        }
        team_sync();
        BPROF(9)  // S-update operands
        team_qr<RS, n, 0, TEAM>(a, RS, tl, bus);
        if (colx) {
#pragma unroll
          for (int i = 0; i < n; i++) Sreg[i + n * tl] = (i <= tl) ? a[i] : 0.0;
          *lane_at(Sreg + SOFF, 1) = sown;
        }
        team_sync();
      }
      {
        double a = 0.0, b2 = 0.0;
#pragma unroll
        for (int i = 0; i < m; i++) a = fma(d[i], Qu[i], a);
#pragma unroll
        for (int i = 0; i < m; i++) b2 = fma(Ud[i], Ud[i], b2);
        dV0 += a;
        dV1 += 0.5 * b2;
      }
    }
    BPROF(10)  // QR S-update (+ std-path S update)
    if (store_S && colx) {
#pragma unroll
      for (int i = 0; i < n; i++)
        Bf.Sdbg[((size_t)b * N + k) * n * n + i + n * tl] =
            Sreg[i + n * tl];
      Bf.sdbg[((size_t)b * N + k) * n + tl] = sown;
    }
    }
    if (!restart) done = true;
  }
  BPROF(11)
  BPROF_FLUSH
  if (!live) return;
  const bool aborted = (s.flags & TOG_TRAJ_BP_ABORTED) != 0;
  if (!aborted) reg_decrease(P, s);  // regularization_update!(solver, :decrease) (backward_pass.jl:82 / :166)
  if (tl == 0) {
    TrajState& g = Bf.st[b];
    g.rho = s.rho;
    g.drho = s.drho;
    g.flags = s.flags;
    g.dV0 = aborted ? 0.0 : dV0;
    g.dV1 = aborted ? 0.0 : dV1;
    g.bp_restarts = restarts + (faithful ? 1 : 0);
    if (aborted) g.active = 0;  // no forward pass, no bookkeeping: the trajectory is finished
  }
}
#undef Eg
#undef ABg
#undef Kg
#undef dg
#undef Qs

}  // namespace tog
