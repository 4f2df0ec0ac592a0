// Internal device interface: POD argument blocks and host-side launchers of
// the HIP kernels (assembly.hip, linalg.hip). Host orchestration code
// (api.cpp, solver.cpp) talks to the GPU only through these functions.
#pragma once
#include <vector>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace dcp {

#define DCP_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) throw dcp::DeviceError(#expr, _e, __FILE__, __LINE__);   \
  } while (0)

struct DeviceError {
  const char* what_expr;
  hipError_t code;
  const char* file;
  int line;
  DeviceError(const char* w, hipError_t c, const char* f, int l)
      : what_expr(w), code(c), file(f), line(l) {}
};

// Node-local constraint form of a velocity support point (the only shapes the
// shell produces: homogeneous no-slip and no-normal-flux, both of which only
// couple the 3 components of one node):
//   type 0: unconstrained; 1: all 3 components fixed to 0;
//   2: component k = sum_{d != k} w[d] u_d.
struct NodeConstraint {
  double w[3];
  int32_t type;
  int32_t k;
};

struct PhysicsDev {
  double dt;            // time_step
  double nu_sys;        // dt/Re: dt*(1/Re)*2*(eps:eps) = dt/Re*(delta grad.grad + d_c' s_a d_c s_b)
  double nu_pre;        // dt/Re: preconditioner dt*(1/Re)*(grad:grad)
  double beta, T_ref;
  double grav_scale, g;
  double coriolis_z;    // (L/U) * omega on the cuboid, else 0 (Q2)
  double one_over_peclet;
  double dt_T;          // dt / NSE_solver_interval (Q8)
  int cuboid;
};

// Per-cell maps into the block-sparse global matrices (absolute entry index).
struct ScatterMaps {
  const int32_t* posA;   // [n_cells][27*27]  A block index of (a, b)
  const int32_t* posBt;  // [n_cells][27*8]   Bt entry of (a, v)
  const int32_t* posB;   // [n_cells][8*27]   B entry of (v, a)
  const int32_t* posT;   // [n_cells][tdpc*tdpc] T CSR entry of (i, j)
};

struct CellData {
  int n_cells;
  const int32_t* cell_q2;   // [n_cells][27] vnode ids (lexicographic)
  const int32_t* cell_p;    // [n_cells][8]  pressure dofs (vertex order)
  const int32_t* cell_T;    // [n_cells][tdpc] temperature dofs (FE_Q(2): lexicographic)
  int tdpc;                 // 8 (FE_Q(1)) or 27 (FE_Q(2)) temperature dofs per cell
  const double* geo;        // [n_cells][64][3] MappingQ(3) support points (fe_tables.h)
  const NodeConstraint* vcon;  // [n_vnodes]
  const uint8_t* T_fixed;   // [n_T] 1 = Dirichlet
  const double* T_bc;       // [n_T] inhomogeneity (valid where T_fixed)
  const double* diameter;   // [n_cells]
  // periodic identification: the cell maps above hold the partner of an
  // identified dof; these hold the original dofs (null when none identified)
  const int32_t* cell_q2o;  // [n_cells][27]
  const int32_t* cell_po;   // [n_cells][8]
  const int32_t* cell_To;   // [n_cells][8]
  // radially separable mesh (X(a,b,c) = r_c phi_ab, api.cpp separable_geometry;
  // null otherwise): J^-1 / JxW / x at the Gauss points from per-column and
  // per-layer tables instead of the MappingQ(3) sums over 64 support points
  const int32_t* sep_col;      // [n_cells]
  const double* sep_colgeo;    // [n_cols][9 points q0 + 3 q1][m0 m1 m2 (/D2), D2]
  const double* sep_colphi;    // [n_cols][9][3] phi at the points
  const int32_t* sep_layer;    // [n_cells]
  const double* sep_laygeo;    // [n_layers][3 points q2][1/R, 1/R', R^2 R']
  const double* sep_layR;      // [n_layers][3] R
};

struct NseOut {
  double* A;     // [nnzb_A][9] or null
  double* Bt;    // [nnz_Bt][3] or null
  double* B;     // [nnz_B][3]  or null
  double* rhs;   // velocity block of nse_rhs or null
  double* elemK; // element mode: [n][89][89]
  double* elemF; // element mode: [n][89]
  // assembled diagonal of the constrained velocity rows, [n_con_nodes][3]
  // (component c of constrained node n at 3 cidx[n] + c), or null
  double* cdiag;
  const int32_t* cidx;  // [n_vnodes] constrained-node index or -1
  // the same for the identified (periodic) pressure dofs: [n_p] index or -1
  double* pcdiag;
  const int32_t* pcidx;
  // k_nse_rhs_halfwave over one list of cells (the cells with a constrained
  // node, colour order): each (list cell k, node t) of a constrained node
  // stores its |K_ii| triple at cbuf[3 cslot[27 k + t]] instead of adding into
  // cdiag; con_gather then sums them per node in list order (null: add)
  double* cbuf = nullptr;
  const int32_t* cslot = nullptr;
};
// cdiag[3 i + c] = sum over slots [cptr[i], cptr[i + 1]) of cbuf[3 slot + c]
void con_gather(int n_con, const int32_t* cptr, const double* cbuf, double* cdiag, hipStream_t s);
// the constrained-row diagonals in Kronecker form (kernels/assembly.hip,
// k_cdk_*): the lateral (10 per column id and lateral node) and radial (4 per
// layer and radial node) tables at upload; per assembly the sums over each
// constrained node's slots [cptr[i], cptr[i + 1]), rec holding per slot the
// pair (lateral table index, radial table index), mask[i] the node's
// constrained components (bit d)
void cdk_tables(const double* colgeo, int n_cols, const double* laygeo, int n_layers, double* L,
                double* R, hipStream_t s);
void cdk_diag(int n_con, const int32_t* cptr, const int32_t* rec, const int32_t* mask,
              const double* L, const double* R, double nu, double* cdiag, hipStream_t s);

// ---- assembly2d.hip -----------------------------------------------------------
// Two-dimensional model (Standard::BoussinesqModel<2>): 22-dof cells over a
// scalar CSR nse_matrix [u | p]; node-local constraint table per cell.
struct Mesh2DDev {
  int n_cells, n_u, tdpc;
  const int32_t* dofs;      // [n_cells][22] FESystem local order
  const int32_t* tdofs;     // [n_cells][tdpc] FE_Q local order
  const double* X;          // [n_cells][16][2] MappingQ(3) support points
  const double* diameter;   // [n_cells]
  const int8_t* src;        // [n_cells][22] constrained local dof whose line targets this one, or -1
  const double* srcw;       // [n_cells][22] its weight
  const uint8_t* fixed;     // [n_cells][22] local dof constrained
  const int32_t* pos;       // [n_cells][22][22] CSR entry of (dof_i, dof_j) or -1
  const int32_t* posT;      // [n_cells][tdpc][tdpc]
  const uint8_t* T_fixed;   // [n_T]
  const double* T_bc;       // [n_T]
};
void launch2d_nse_system(const Mesh2DDev& m, const int32_t* cells, int n, const double* old_nse,
                         const double* old_T, const PhysicsDev& ph, double* A, double* rhs,
                         hipStream_t s);
void launch2d_nse_elements(const Mesh2DDev& m, int first, int n, const double* old_nse,
                           const double* old_T, const PhysicsDev& ph, double* K, double* f,
                           hipStream_t s);
void launch2d_precond_diag(const Mesh2DDev& m, const int32_t* cells, int n, const PhysicsDev& ph,
                           double* Ad, double* Mpd, hipStream_t s);
void launch2d_T_matrix(const Mesh2DDev& m, const int32_t* cells, int n, const PhysicsDev& ph,
                       double* M, double* K, hipStream_t s);
void launch2d_T_rhs(const Mesh2DDev& m, const int32_t* cells, int n, const double* T_old,
                    const double* nse, const PhysicsDev& ph, double* rhs, hipStream_t s);
void velocity_stats_2d(const Mesh2DDev& m, const double* nse, double* out2, hipStream_t s);
void distribute_2d(int n_lines, const int32_t* line_dof, const int32_t* ptr, const int32_t* ent,
                   const double* w, const double* inhom, double* x, hipStream_t s);
void positions_2d(int n_cells, int dpc, const int32_t* dofs, const int32_t* ptr, const int32_t* col,
                  int32_t* pos, hipStream_t s);

// ---- matfree.hip ----------------------------------------------------------
// Matrix-free [A B^T; B 0] (or A alone) of the classic Q2^3/Q1 system.
// Per-cell arrays in colour order (position e = e-th cell of the colour-sorted
// cell list).
struct MfData {
  int n_u;                     // offset of the pressure block in [u | p]
  const int32_t* cell_q2;      // [n_cells][27]
  const int32_t* cell_p;       // [n_cells][8]
  const NodeConstraint* vcon;  // [n_vnodes]
  const double* geo;           // [n_cells][10][27]: J^-1 (9), JxW
  const uint64_t* first;       // [n_cells] first-touch bits: node t -> bit t,
                               // pressure vertex v -> bit 32 + v
};
void mf_geometry(const CellData& cd, const int32_t* order, double* geo, hipStream_t s);

// Cell-order matrix-free apply (two launches, no colouring):
//   k_mf_pencil: every cell (tree order) evaluates K_cell C x with its geometry
//     from the radially separable tables (or the streamed per-point J^-1 /
//     JxW of a general mesh) and stores its 27 velocity
//     triples and 8 pressure values to their slots in the dof-sorted
//     incidence list (slot of (cell, t) = rank of the cell among the cells of
//     node t, ascending cell order);
//   k_mf_gather: every dof sums its contiguous run of slots in that order
//     (deterministic), applies C^T and the constrained diagonal.
// Workgroup b runs on XCD b % 8 (round-robin dispatch). This bijection gives
// each XCD one contiguous range of logical blocks, so neighbouring cells (which
// share nodes) meet in the same L2.
__device__ inline int xcd_block(int b, int G) {
  const int q = G >> 3, r = G & 7, x = b & 7, i = b >> 3;
  return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}
#ifndef DCP_MF_WAVES
#define DCP_MF_WAVES 1
#endif
// chain links of the velocity partial sums inside a cell group (27 per cell)
using MfLink = std::conditional_t<(27 * 7 * DCP_MF_WAVES < 255), uint8_t, uint16_t>;
constexpr MfLink kMfLinkEnd = MfLink(~MfLink(0));
struct MfCells {
  int n_cells;
  int n_u;                     // offset of the pressure block in [u | p]
  const int32_t* cell_q2;      // [n_cells][27] (tree order)
  const int32_t* cell_p;       // [n_cells][8]
  const double* geo;           // [n_cells][10][27] J^-1 / JxW (non-separable meshes only)
  const NodeConstraint* vcon;  // [n_vnodes]
  const uint32_t* cmask;       // [n_cells] bit t: local node t is constrained
  // Velocity records are summed per cell group (kMfGroupCells consecutive
  // cells from the launch's first cell, one wave) before they leave the
  // kernel: the first occurrence of a node in its group owns the group's
  // partial sum, the later ones are chained to it in (cell, t) order.
  const int32_t* vslot;        // [n_cells][27] buf offset (doubles) of the owner's partial, or -1
  const MfLink* vnext;         // [n_cells][27] next occurrence in the group (27 * cell + t), or kMfLinkEnd
  const int32_t* pslot;        // [n_cells][8]  buf offset of the (cell, v) pressure value
  // Radially separable geometry (null if the mesh is not): X(a,b,c) = r_c phi_ab
  // in every cell, so J^-1 / JxW at a Gauss point follow from a per-column 2D
  // table and the cell's three node-layer radii (see mf_separable_geometry).
  const int32_t* col;          // [n_cells] column of the cell
  const double* colgeo;        // [n_cols][9 points q0 + 3 q1][m0 m1 m2 D2] (10)
  const int32_t* layer;        // [n_cells] radial layer of the cell
  const double* laygeo;        // [n_layers][3 points][1/R, 1/R', R^2 R']
  // the NSE rhs in cell order (mf_rhs): temperature dofs, the lateral
  // directions Phi at the 9 column points and the layer radii R at the 3
  // radial points (x = R Phi)
  const int32_t* cell_T = nullptr;  // [n_cells][8]
  const double* colphi = nullptr;   // [n_cols][9][3]
  const double* layR = nullptr;     // [n_layers][3]
  const double* colphin = nullptr;  // [n_cols][9][|Phi|, 1/|Phi|, 1/sqrt|Phi|]
  const double* layRs = nullptr;    // [n_layers][3] sqrt(R)
};
struct MfGather {
  int n_vnodes, n_p, n_u;
  // dofs in gather order (by the chunk of their last cell, then id): position
  // i is velocity node vorder[i] / pressure dof porder[i]
  const int32_t* vorder;
  const int32_t* porder;
  const int32_t* vptr;         // [n_vnodes + 1] slot ranges per position: triples buf[3 k .. 3 k + 2]
  const int32_t* pptr;         // [n_p + 1] slot ranges per position: buf[pbase + k]
  int32_t pbase;               // 3 * vptr[n_vnodes]
  const int32_t* cidx;         // [n_vnodes] constrained-node index or -1
  const NodeConstraint* vcon;
  const double* cdiag;         // [n_con_nodes][3] assembled diagonal (NseOut::cdiag)
  const int32_t* pcidx;        // [n_p] identified pressure dof index or -1 (null: none)
  const double* pcdiag;        // their assembled diagonal
  // [ceil(n_vnodes / 64)]: 1 if positions [64 b, 64 b + 64) hold a
  // constrained node (null: always look cidx up)
  const uint8_t* wcon;
};
// waves per workgroup of k_mf_pencil (7 cells each); the workgroup's cells
// are the cell group of the velocity partial sums
constexpr int kMfGroupCells = 7 * DCP_MF_WAVES;
// cells [c0, c1) / gather positions [v0, v1) and [p0, p1)
void mf_cells(const MfCells& mc, int c0, int c1, double nu, bool stokes, const double* src,
              double* buf, double* dst, hipStream_t s);
// The fused apply's schedule (k_mf_fused, built at upload): per workgroup a
// task (kind << 30 | index; kind 0 pencil batch, 1 velocity window, 2
// pressure window, 3 padding); per gather window (velocity windows first) the
// pencil batches whose records it reads (dep_ptr / dep); done[batch] = the
// apply's seq once the batch's records are stored; err (host-mapped) set
// when a poll exceeded spin_limit.
struct MfFused {
  const int32_t* sched;
  const int32_t* dep_ptr;
  const int32_t* dep;
  unsigned* done;
  double* err;
  int n_vwin;
  long spin_limit;
};
void mf_fused(const MfCells& mc, const MfGather& mg, const MfFused& f, int n_tasks, double nu,
              bool stokes, const double* src, double* buf, double* dst, unsigned seq,
              hipStream_t s);
// the NSE rhs (mf_rhs_cells + the velocity gather with condensation only, mg.cdiag
// null) in the same one-launch form
void mf_rhs_fused(const MfCells& mc, const MfGather& mg, const MfFused& f, int n_tasks,
                  const double* u_old, const double* T_old, const PhysicsDev& ph, double* buf,
                  double* rhs, unsigned seq, hipStream_t s);
void mf_gather(const MfGather& mg, int v0, int v1, int p0, int p1, bool stokes, const double* buf,
               const double* src, double* dst, hipStream_t s);
// The velocity rhs of local_assemble_nse_system (boussinesq_model.tpp:655-669)
// in cell order (separable shell or cuboid, FE_Q(1) temperature): the pencil
// kernel with the rhs flux per point into the velocity records of buf (cells
// [c0, c1), one chunk of the cell-order layout), then mf_gather of the
// velocity positions with mg.cdiag = null (condensation only) into rhs[0, n_u)
void mf_rhs_cells(const MfCells& mc, int c0, int c1, const double* u_old, const double* T_old,
                  const PhysicsDev& ph, double* buf, double* rhs, hipStream_t s);
// one colour class = positions [base, base + n): dst (+)= C^T K C src
void mf_apply_colour(const MfData& md, int base, int n, double nu, bool stokes,
                     const double* src, double* dst, hipStream_t s);
// constrained velocity dofs: dst[dof] = cdiag[diag_pos] * src[dof]
void mf_constrained(int n, const int32_t* dof, const int64_t* diag_pos, const double* cdiag,
                    const double* src, double* dst, hipStream_t s);

// ---- assembly.hip ---------------------------------------------------------
// Colour-wise NSE system assembly (cells of one colour share no node, so the
// read-modify-write scatter needs no atomics and is deterministic). mfma: the
// velocity-block Gram sums on v_mfma_f64_16x16x4_f64 (DCP_OPT_ELEMENT_MFMA).
void launch_nse_system(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                       const double* u_old, const double* T_old, const PhysicsDev& ph,
                       const NseOut& out, hipStream_t s, bool mfma = false);
// Operator form (out.A ignored): B^T, B, rhs and out.cdiag; the velocity
// block stays matrix-free.
void launch_nse_operator(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                         const double* u_old, const double* T_old, const PhysicsDev& ph,
                         const NseOut& out, hipStream_t s);
// dst block k (3 doubles) = src block tperm[k]: B from B^T (operator form)
void transpose_blocks3(long n, const int32_t* tperm, const double* src, double* dst,
                       hipStream_t s);
// Element mode: dense FESystem-ordered K/f of cells [first, first+n).
void launch_nse_system_elements(const CellData& cd, int first, int n, const double* u_old,
                                const double* T_old, const PhysicsDev& ph, double* K, double* f,
                                hipStream_t s, bool mfma = false);
void launch_nse_precond_diag(const CellData& cd, const int32_t* cells, int n, const PhysicsDev& ph,
                             double* A_diag, double* Mp_diag, hipStream_t s);
// posTs: [n_cells][8] position of (original, original) for identified T dofs, -1 else (or null)
void launch_T_matrix(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                     const PhysicsDev& ph, double* Tmass, double* Tstiff, const int32_t* posTs,
                     hipStream_t s);
// A(s,s) block of every identified velocity node s = diag(cdiag of s)
void image_diagonal_blocks(int n, const int32_t* node, const int64_t* blk, const int32_t* cidx,
                           const double* cdiag, double* A_val, hipStream_t s);
// FE_Q(2) temperature (kernels/temperature_q2.hip); launch_T_matrix / launch_T_rhs
// dispatch to these when cd.tdpc == 27
void launch_T2_matrix(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                      const PhysicsDev& ph, double* Tmass, double* Tstiff, hipStream_t s);
void launch_T2_rhs(const CellData& cd, const int32_t* cells, int n, const double* T_old,
                   const double* u_cur, const PhysicsDev& ph, double* rhs, hipStream_t s);
void launch_T_rhs(const CellData& cd, const int32_t* cells, int n, const double* T_old,
                  const double* u_cur, const PhysicsDev& ph, double* rhs, hipStream_t s);

// Temperature system on a radially separable mesh that is the full product of
// columns and layers (kernels/temperature_sep.hip: Kronecker-form assembly; tsep.cpp
// builds the tables at upload).
struct TSepDev {
  int n_colids = 0;   // column ids of the separable geometry (mapping kinds apart)
  int n_layers = 0;   // radial layers; levels 0..n_layers
  int n_kinds = 0;    // mapping kinds of the layers
  int n_latnnz = 0;   // entries of the lateral pattern
  const double* colgeo = nullptr;   // separable tables (CellData::sep_*)
  const double* laygeo = nullptr;
  const double* layR = nullptr;
  const int32_t* ord2lay = nullptr;  // [n_layers] layer id of radial ordinal o
  const int32_t* lay2ord = nullptr;  // [layer ids] ordinal
  const int32_t* kind = nullptr;     // [n_layers] mapping kind of ordinal o
  int n_con = 0;                     // lateral contributions (per kind)
  int probe = 0;                     // DCP_TSEP_PROBE timing variants (0: the real kernels)
  const int32_t* lptr = nullptr;     // [n_latnnz + 1]
  const int32_t* lcon = nullptr;     // [n_kinds][n_con] column id << 4 | alpha << 2 | beta
  const uint16_t* cmask = nullptr;   // [n_cells] fixed vertices | lifted vertices << 8
  const uint32_t* code = nullptr;    // [nnz of T] (k_tsep_matrix)
  // k_tsep_matrix_lds: per block of blk_pt x 256 consecutive entries its
  // distinct A records (kind n_latnnz + p), staged in LDS; the entries coded
  // by slot (bits 0-9 term a, 10-19 term b, 20-27 l, 28-29 dl, 30 zero, 31
  // diagonal) in rcode. blk_pt 0: no lists (k_tsep_matrix reads A per entry)
  int blk_pt = 0, max_rec = 0;
  const int32_t* blk_ptr = nullptr;
  const int32_t* blk_rec = nullptr;
  const uint32_t* rcode = nullptr;
  const int32_t* T_col = nullptr;
  const int32_t* sptr = nullptr;     // [n_T + 1] records of each T dof
  const int32_t* slot = nullptr;     // 8 cell + a, ascending cell
  double* loc = nullptr;             // [n_colids][64] lateral tables
  double* rad = nullptr;             // [n_layers][16] radial tables
  double* A = nullptr;               // [n_kinds][n_latnnz][6] (M, ll, x, x^T, 22, pad)
  double* rec = nullptr;             // [n_cells][8] rhs records
};
// the lateral / radial tables of the column ids and layers (mesh geometry,
// formed once at upload like the B^T column / layer factors)
void tsep_tables(const TSepDev& t, hipStream_t s);
// B^T in Kronecker form (kernels/bt_kron.hip; btkron.cpp builds the tables).
// k_btk_entries: one workgroup of kBtkTB threads per kBtkPT * kBtkTB
// consecutive entries; btkron.cpp lists each such block's distinct lateral
// records (kind, pair), staged into LDS, and codes the entries by slot.
#ifndef DCP_BTK_PT
#define DCP_BTK_PT 8
#endif
constexpr int kBtkTB = 256;
constexpr int kBtkPT = DCP_BTK_PT;
constexpr long kBtkBlock = long(kBtkPT) * kBtkTB;
constexpr int kBtkMaxRec = 1023;  // slots per block (10-bit slot fields of the code)
struct BtkDev {
  int n_layers = 0, n_kinds = 0, n_pairs = 0, n_con = 0, n_conent = 0;
  int max_rec = 0;                   // largest record list of a block
  const double* P = nullptr;         // column factors (k_bt_coltab)
  const double* Q = nullptr;         // layer factors by layer id (k_bt_laytab)
  const int32_t* ord2lay = nullptr;  // [n_layers]
  const int32_t* kind = nullptr;     // [n_layers] mapping kind of ordinal layer
  const int32_t* lptr = nullptr;     // [n_pairs + 1] lateral (node, vertex) pairs
  const int32_t* lcon = nullptr;     // [n_kinds][n_con] offset of the pair's P entry
  // per entry: slot of the first term (bits 0-9), of the second (10-19),
  // node level lambda (20-27), l - lambda / 2 + 1 (28-29), constrained row
  // (30; then the slot field of the absent term holds the row's index in the
  // block's constrained rows)
  const uint32_t* code = nullptr;      // [nnz of B^T]
  const int32_t* blk_ptr = nullptr;    // [blocks + 1] record lists
  const int32_t* blk_rec = nullptr;    // records kind n_pairs + pair
  const int32_t* blk_cptr = nullptr;  // [blocks + 1] constrained rows of each block
  const int32_t* blk_crow = nullptr;  // their row (velocity node) ids
  int max_con = 0;                    // largest such list
  double* A = nullptr;               // [n_kinds][n_pairs][6]
};
void btk_assemble(const BtkDev& b, long nnz, const NodeConstraint* vcon, double* Bt,
                  hipStream_t s);
// M, K, T_matrix = M + dt_T K and its Jacobi inverse (every entry written)
void tsep_matrix(const TSepDev& t, long nnz, const PhysicsDev& ph, double* M, double* K,
                 double* Tmat, double* Tinv, hipStream_t s);
// the temperature rhs (overwritten; needs tsep_matrix's tables)
void tsep_rhs(const TSepDev& t, const CellData& cd, int n_T, const double* T_old,
              const double* u, const PhysicsDev& ph, double* rhs, hipStream_t s);
// Builds posA/posBt/posB/posT by binary search in the sorted patterns.
void launch_build_scatter_maps(const CellData& cd, const int32_t* A_ptr, const int32_t* A_col,
                               const int32_t* Bt_ptr, const int32_t* Bt_col, const int32_t* B_ptr,
                               const int32_t* B_col, const int32_t* T_ptr, const int32_t* T_col,
                               int32_t* posA, int32_t* posBt, int32_t* posB, int32_t* posT,
                               hipStream_t s);

// Re-encode the scatter positions of the first cell (in colour launch order)
// touching each block as ~pos; true if every one of the nnz blocks is touched
// (then the assembly stores first and needs no zero fill), else the
// positions are left plain.
// B^T of the operator-form assembly on the radially separable shell
// (assembly.hip k_bt_coltab + k_bt_tasks): P = [n_cols][216] column factors
// and Q = [n_layers][12] layer factors, formed when n_cols / n_layers > 0
// (once, at upload: geometry only);
// task_hdr [n_tasks][4] / slot_rec [slots][4]: runs of consecutive velocity
// node rows (<= 8 (row, cell) slots, <= 64 entries) built at upload
// (api.cpp build_bt_tasks). Writes every B^T entry once; B is read as its
// transpose (the row tasks are used only where every local B entry has its
// B^T entry, Ctx::B_transpose).
void launch_bt_rows(const CellData& cd, int n_cols, int n_layers, double* P, double* Q,
                    int n_tasks, int slots, const int32_t* task_hdr, const int32_t* slot_rec,
                    double* Bt, hipStream_t s);
bool mark_first_touch(const int32_t* color_cells, const std::vector<int>& color_ptr, int per_cell,
                      int32_t* pos, size_t n_cells, size_t nnz, hipStream_t s,
                      unsigned long long* touched_out = nullptr);

// S = B diag(d) B^T into the precomputed CSR pattern (one wavefront per row,
// contributions summed in fixed node order: deterministic). pmap != null:
// entry j of the CSR pattern is stored at S_val[pmap[j]] (the SELL layout).
// B_val == null: B[p][n] read as B^T block tperm[k] (B not materialised)
void form_schur_complement(int n_p, const int32_t* B_ptr, const int32_t* B_col, const double* B_val,
                           const int32_t* tperm, const int32_t* Bt_ptr, const int32_t* Bt_col,
                           const double* Bt_val,
                           const double* d, const int32_t* S_ptr, const int32_t* S_col,
                           const int32_t* pmap, double* S_val, int max_row, hipStream_t s);

// ---- ilu.hip ------------------------------------------------------------------
// ILU(0) of nse_matrix.block(0,0) on its scalar pattern (Schur-complement
// solver). ptr/col/diag: scalar CSR of the block-CSR A (pos[k]: A_val index of
// entry k); lf_*: row levels of the factorisation / forward solve, lb_*: of
// the backward solve.
struct IluView {
  int n;
  long nnz;
  const int32_t *ptr, *col, *diag, *pos;
  int n_lf, n_lb;
  const int32_t *lf_ptr, *lf_rows, *lb_ptr, *lb_rows;
};
// max_row: the longest scalar row (a wave per row staged in LDS up to 512)
void ilu_factor(const IluView& f, const double* A_val, const int* lf_host_ptr, double* lu,
                int max_row, hipStream_t s);
void ilu_apply(const IluView& f, const double* lu, const double* b, double* x, hipStream_t s);
void zero_at(int n, const int32_t* idx, double* x, hipStream_t s);

// ---- linalg.hip -------------------------------------------------------------
// y (=|+=) alpha * M x for block-CSR with R x C blocks (R,C in {1,3}).
void spmv_bsr33(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                const double* x, double* y, bool add, hipStream_t s);
void spmv_bsr31(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                const double* x, double* y, bool add, hipStream_t s);
void spmv_bsr13(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                const double* x, double* y, bool add, hipStream_t s);
void spmv_csr(int rows, const int32_t* ptr, const int32_t* col, const double* val,
              const double* x, double* y, bool add, hipStream_t s);
// CSR with long rows (~125 nnz, the Schur complement): 32 lanes per row
void spmv_csr_long(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                   const double* x, double* y, bool add, hipStream_t s);

// SELL-64 SpMV: slices of 64 consecutive rows (one wave, one row per lane);
// slice width even; inside a slice entries are stored in column pairs (row
// 64s+i, entry k at off[s] + 128 (k/2) + 2i + k%2; padding: col = own row,
// val = 0), so a lane reads two entries with one 16-B (values) / 8-B or 4-B
// (columns) load and every load of a wave is one contiguous segment. Columns
// are 32-bit (col) or 16-bit offsets from a per-slice base (col16 + base).
//   y = M (cf * x)
__host__ __device__ inline int64_t sell_pos(const int64_t* off, int p, int k) {
  return off[p >> 6] + 128 * int64_t(k >> 1) + 2 * (p & 63) + (k & 1);
}
struct SellView {
  int rows;
  const int64_t* off;
  const int32_t* col;      // or null
  const uint16_t* col16;   // with base, or null
  const int32_t* base;
  const double* val;
  const int32_t* rowmap = nullptr;  // row -> vector entry (null: the row itself)
  // structured columns (one GPU, radially layered shell; col / col16 null):
  // row r = level l * nc + lateral c, with nd = the levels of [l - 2, l + 2]
  // inside [0, nl) from l + dlo on, entry k = nd j + d of the row is column
  // (l + dlo + d) nc + nbr[min(j, nj - 1) nc + c] (entries past the row's own
  // neighbour count hold value 0; table row nj - 1 is the lateral itself)
  const int32_t* nbr = nullptr;
  int nc = 0, nl = 0, nj = 0;
};
void sell_spmv(const SellView& m, const double* x, double cf, double* y, hipStream_t s);
// y = (S x - theta x) * sscale (the s-step Newton basis); every launch returns
// at entry once *status != 0
void sell_spmv_shifted(const SellView& m, const double* x, double theta, double sscale, double* y,
                       const int* status, hipStream_t s);
// *out = max_i sum_j |S_ij| (Gershgorin bound of the spectrum of S)
void sell_gershgorin(const SellView& m, double* out, hipStream_t s);
// Krylov-fused form: additionally xs = cf * x on every row (the scaled basis
// vector, xs != x), and per-workgroup partials of y.v0 -> part0 and y.y ->
// part1 (one per slice, fixed order; zeros up to n_part, the length common to
// all ranks whose partials are all-reduced).
// Per-step block of the inner Schur GMRES with modified Gram-Schmidt
// (solver.cpp): [0, 128) coefficients h_0.., kSpNStart the start norm of the
// loss-of-orthogonality test, the chain's final partials from kSpPart.
constexpr int kSpNStart = 128, kSpPart = 192;
int sell_fused_blocks(int rows);
void sell_spmv_fused(const SellView& m, const double* x, double cf, double* xs, double* y,
                     const double* v0, double* part0, double* part1, int n_part, hipStream_t s);
// Step of the device-resident GMRES cycle: y = M (cf * x) with cf = *cf_dev
// (cf_dev null: 1), xs = cf * x when xs != null; nothing if *status != 0.
void sell_spmv_step(const SellView& m, const double* x, const double* cf_dev, double* xs,
                    double* y, const int* status, hipStream_t s);

// Scalars live in device memory ("device scalars") so Krylov kernels can
// chain without host round trips. A coefficient argument is (ptr, mult):
// value = mult * (ptr ? *ptr : 1).
struct DScal {
  const double* p;
  double m;
};
// Owned part of a local vector for reductions: entries [0, n1),
// [off2, off2 + n12 - n1) and [off3, off3 + n - n12). The multi-GPU NSE
// layout [u_own u_ghost | p_own p_ghost] has two owned segments, the FEEC one
// [w_own w_ghost | u_own u_ghost | p_own p_ghost] three; every other vector
// (and every single-GPU vector) is a prefix, Seg::all(n).
struct Seg {
  int n1, off2, n12, off3, n;
  int kind;  // vector family (chain width selection on several GPUs), -1: any
  static Seg all(int n, int kind = -1) { return Seg{n, 0, n, 0, n, kind}; }
  static Seg two(int n1, int off2, int n, int kind) { return Seg{n1, off2, n, 0, n, kind}; }
};
// Partial-sum reduction buffer: kReduceBlocks doubles per slot.
constexpr int kReduceBlocks = 512;
// dot(a,b) -> *out (two launches, deterministic order)
void dot(Seg g, const double* a, const double* b, double* partials, double* out, hipStream_t s);
// partials only (kReduceBlocks of them) / the final fixed-order sum
void dot_partials(Seg g, const double* a, const double* b, double* partials, hipStream_t s);
void reduce_final(int nb, const double* partials, double* out, hipStream_t s);
// v += c * x; then *out = v . w (w == v allowed) — deal.II add_and_dot
void add_and_dot(Seg g, double* v, DScal c, const double* x, const double* w, double* partials,
                 double* out, hipStream_t s);
void add_and_dot_partials(Seg g, double* v, DScal c, const double* x, const double* w,
                          double* partials, hipStream_t s);
// Launch-lean Gram-Schmidt chain (one launch per step, no reduction launches):
//   dot_partial writes nb block sums of a.b; chain_add_and_dot reduces the
//   previous step's nb partials (stores the sum to *coef_store from block 0),
//   does v += mult * sum * x and writes the nb partials of v.w.
constexpr int kChainMaxBlocks = 1024;
int chain_blocks(int n);
void dot_partial(Seg g, const double* a, const double* b, double* partials, int nb, hipStream_t s);
void chain_add_and_dot(Seg g, double* v, const double* prev, double mult, const double* x,
                       const double* w, double* partials, double* coef_store, int nb,
                       hipStream_t s);
// Same step with nb_prev previous partials (e.g. from sell_spmv_fused), an
// optional second partial array prev2 whose fixed-order sum block 0 stores to
// *store2, and optionally a second copy of the partials (partials_host: mapped
// host memory, so the host reads them without a copy launch).
void chain_add_and_dot_ex(Seg g, double* v, const double* prev, int nb_prev, double mult,
                          const double* x, const double* w, double* partials,
                          double* coef_store, int nb, const double* prev2, double* store2,
                          double* partials_host, hipStream_t s);
// The whole chain in one launch (kernels/linalg.hip k_mgs_chain; one GPU):
// h_0 = w.V[0] (the sum of prev's nb_prev partials, or computed in-kernel when
// prev is null), h_i = (w -= h_{i-1} V[i-1]).V[i], w -= h_{d-1} V[d-1], nb
// partials of |w|^2 -> partials (+ partials_host); h_0..h_{d-1} -> coef.
// Bitwise the per-step chain above. Needs every one of the nb workgroups
// resident: mgs_chain_fits() says whether (n, nb, d) qualify on n_cus CUs.
// gran: kMgsGranules doubles of hand-off scratch; seq: a per-context launch
// counter (never reused); *err becomes 1 if a workgroup timed out waiting.
constexpr int kMgsMaxVecs = 64;
constexpr size_t kMgsGranules = size_t(2) * kMgsMaxVecs * kChainMaxBlocks;
struct ChainVecs {
  const double* v[kMgsMaxVecs];
};
bool mgs_chain_fits(long n, int nb, int d, int n_cus);
void mgs_chain(Seg g, double* w, const ChainVecs& V, int d, const double* prev, int nb_prev,
               const double* prev2, double* store2, double* coef, double* partials,
               double* partials_host, int nb, double* gran, unsigned long long seq, double* err,
               hipStream_t s);
// ---- krylov.hip: device-resident GMRES cycle with classical Gram-Schmidt twice
// State of one restart cycle of deal.II SolverGMRES kept in device memory: the
// Hessenberg columns, Givens rotations, residual estimates and the
// SolverControl decision (status 0: iterate, 1: success, 2: failure).
constexpr int kGmMaxDim = 32;
struct GmresDev {
  double H[kGmMaxDim][kGmMaxDim];   // rotated columns (R of the Givens QR), back substitution
  double gamma[kGmMaxDim + 1], ci[kGmMaxDim], si[kGmMaxDim];
  double coef[2 * kGmMaxDim];   // this step's first / second pass coefficients
  double y[kGmMaxDim];          // back-substituted combination coefficients
  double inv_norm, rho, tol;    // 1/|w| of the last step (1 if 0), |gamma_dim|, tolerance
  double nrm2;                  // |w|^2 of the last step
  double inv_rho;               // 1 / the residual norm at the start of the cycle
  int status, dim, accumulated, max_steps;
  // DCGS2 (one reduction per step, delayed re-orthogonalisation): the raw
  // Hessenberg columns (provisional column k until step k + 1 corrects it)
  // and the pending scale nu_k / beta_k of that correction
  double Hr[kGmMaxDim + 1][kGmMaxDim];
  double c_pend;
  // status as the launch before a multi-launch step's last kernel saw it: that
  // kernel's block 0 may stop the cycle (Givens step) while its other blocks
  // still have their rows to write, so they test this copy, not status
  int status_in;
};
// What the host reads after a cycle (pinned, written by gmres_cycle_end)
struct GmresReport {
  double rho;
  int status, accumulated;
};
struct Comm;
// Arnoldi step k = d - 1 after w = S v_k: w -= V (V^T w) twice, |w|, the
// Givens update and the convergence check (every launch returns at entry once
// st->status != 0). gran: cgs2_granules(g.n) doubles of hand-off granules;
// cnt: a zeroed device counter; seq: the context's launch counter (granule
// tags, never reused); err: set to 1 if a reduction timed out; comm: all-reduce
// the sums (several GPUs) or null.
size_t cgs2_granules(long n);
// s-step Arnoldi block (kernels/krylov.hip k_sstep_block): the raw Newton
// basis w[0..s) (w_i = (S - theta_i) w_{i-1} * (1/sigma), w_0 = q_k) is
// orthogonalised against q_0..q_k twice and Cholesky-QR'd into q[0..s) =
// q_{k+1..k+s}; workgroup 0 forms Hessenberg columns k..k+s-1 and runs their
// Givens steps / checks. One GPU, nb resident workgroups as cgs2_chain_step.
constexpr int kSStep = 4;
struct SStepArgs {
  const double* w[kSStep];
  double* q[kSStep];
  double theta[kSStep];
  double sigma;
};
// co-resident workgroups of the one-launch s-step block (resident.h)
int sstep_block_capacity();
void sstep_block(Seg g, const ChainVecs& V, const SStepArgs& a, int k, GmresDev* st, double* gran,
                 int nb, unsigned long long seq, double* err, hipStream_t s);
// Several GPUs / large meshes: the same block as five launches (dots, column
// sums, dots, column sums, final) around two all-reduces of the per-rank sums (c1: s (k+1) doubles, c2: s (k+1) + s (s+1) / 2; device
// scratch), the reductions over the owned entries of g.
void sstep_block_multi(Seg g, const ChainVecs& V, const SStepArgs& a, int k, GmresDev* st,
                       double* gran, unsigned* cnt, double* c1, double* c2,
                       unsigned long long& seq, double* err, Comm* comm, hipStream_t s);
// One GPU: the same step (w -= V V^T w twice, |w|, Givens) in one launch of
// nb resident workgroups (cgs2_chain_fits: nb <= n_cus, enough entries per
// thread) handing their sums over as granules in gran (kMgsGranules doubles).
bool cgs2_chain_fits(long n, int nb, int n_cus);
// Test hook: the hand-off poll bound of the one-launch CGS2 / DCGS2 / s-step
// kernels (<= 0: the default, kernels/granule.h kMgsMaxSpins).
void set_handoff_spin_limit(long spins);
void cgs2_chain_step(Seg g, double* w, const ChainVecs& V, int d, GmresDev* st, double* gran,
                     int nb, unsigned long long seq, double* err, hipStream_t s);
void cgs2_gmres_step(Seg g, double* w, const ChainVecs& V, int d, double* gran, unsigned* cnt,
                     GmresDev* st, unsigned long long& seq, double* err, Comm* comm,
                     hipStream_t s);
// DCGS2 Arnoldi step k (delayed classical Gram-Schmidt with one global
// reduction per step; Swirydowicz et al. 2020, Bielich et al. 2022) after
// w = S t_k, where t_k = V[k] is the tentative (once orthogonalised) k-th
// basis vector. One reduction gives V_{<k}^T [t w], t.t, t.w, w.w; then
//   q_k = (t_k - V a) / beta, beta = sqrt(t.t - |a|^2)          -> V[k]
//   t_{k+1} = (w - V z - g_k q_k) / nu, nu^2 = w.w - |g|^2      -> tnext
// and the Hessenberg column k - 1 gets its correction (H[:k, k-1] += c a,
// H[k, k-1] = c beta), its Givens rotation and the SolverControl check;
// column k is left provisional. tail (tnext == null, w == null): only the
// correction of column k - 1 (the cycle's last column). One launch of nb
// resident workgroups on one GPU (dcgs2_fits, like cgs2_chain_fits), else
// (several GPUs) partials + last-block reduction, all-reduce, update launch.
bool dcgs2_fits(long n, int nb, int n_cus);
// hand-off granules (doubles) dcgs2_step needs for vectors of n entries
size_t dcgs2_granules(long n);
void dcgs2_step(Seg g, const double* w, const ChainVecs& V, int k, double* tnext, GmresDev* st,
                double* gran, unsigned* cnt, int nb, unsigned long long& seq, double* err,
                Comm* comm, bool one_launch, hipStream_t s);
// Restart-cycle head on the device (SolverGMRES's start of a cycle):
// rho = sqrt(*rho2) of the residual b - S x, SolverControl::check(accumulated,
// rho), gamma_0 = rho, inv_rho = 1 / rho. first: a new solve (tol, max_steps,
// counters reset). Once the solve has stopped (status != 0) it only zeroes
// dim, so every launch of a cycle enqueued after the stop is a no-op.
void gmres_cycle_init(GmresDev* st, const double* rho2, double tol, int max_steps, bool first,
                      hipStream_t s);
// Cycle tail: x += V y (y = the back-substituted coefficients, dim of them,
// read on the device) and the report to the host.
void gmres_cycle_end(GmresDev* st, int n, const double* const* V, double* x, GmresReport* report,
                     hipStream_t s);
// st->y = H^-1 gamma over st->dim
void gmres_backsub(GmresDev* st, hipStream_t s);
// One GPU, S in SELL form: the restart head as two launches. y = b - S x with
// per-slice partials of |y|^2 (sell_spmv_residual), then every workgroup sums
// the partials in the same fixed order, workgroup 0 runs the cycle_init check
// and all scale v0 = y / |y| (gmres_cycle_head).
void sell_spmv_residual(const SellView& m, const double* x, const double* b, double* y,
                        double* part, hipStream_t s);
void gmres_cycle_head(GmresDev* st, const double* part, int n_part, double tol, int max_steps,
                      bool first, int n, const double* p, double* v0, hipStream_t s);
// The restart tail as one launch: every workgroup solves H y = gamma (the
// same arithmetic as k_gmres_backsub), updates its share of x += V y;
// workgroup 0 stores y and the host report.
void gmres_cycle_finish(GmresDev* st, int n, const double* const* V, double* x,
                        GmresReport* report, hipStream_t s);
void axpy(int n, DScal c, const double* x, double* y, hipStream_t s);            // y += c x
void scale(int n, DScal c, double* x, hipStream_t s);                             // x *= c
void sadd(int n, double s_, double a, const double* x, double* y, hipStream_t s); // y = s y + a x
void copy(int n, const double* x, double* y, hipStream_t s);
void equ(int n, DScal c, const double* x, double* y, hipStream_t s);             // y = c x
void axpby(int n, DScal a, const double* x, DScal b, double* y, hipStream_t s);  // y = a x + b y
// *out = *num / *den (one thread)
void scalar_div(const double* num, const double* den, double* out, hipStream_t s);
void fill(int n, double v, double* y, hipStream_t s);
void mul(int n, const double* a, const double* x, double* y, hipStream_t s);     // y = a .* x
void reciprocal(int n, const double* a, double* y, hipStream_t s);                // y = 1/a
// inv[r] = 1 / A(r,r) for a CSR matrix with sorted columns (Ifpack point Jacobi)
void csr_diag_inverse(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                      double* inv, hipStream_t s);
// y = sum_i coef[i] * X[i] (accumulated into y), X given as a device array of pointers
// the same with up to kMgsMaxVecs coefficients and vectors passed by value
struct CombineArgs {
  double c[kMgsMaxVecs];
  const double* x[kMgsMaxVecs];
};
void multi_axpy_args(int n, int k, const CombineArgs& a, double* y, hipStream_t s);
void multi_axpy(int n, int k, const double* coef, const double* const* X, double* y,
                hipStream_t s);
// z = a + alpha * b (elementwise, e.g. T_matrix = M + dt K over one pattern)
void lincomb(int n, const double* a, double alpha, const double* b, double* z, hipStream_t s);
// constraints: velocity distribute (x_k = sum w x_d, Dirichlet -> 0)
void distribute_velocity(int n_vnodes, const NodeConstraint* vcon, double* u, hipStream_t s);
void distribute_temperature(int n_T, const uint8_t* fixed, const double* bc, double* T,
                            hipStream_t s);
// periodic images: x[img[k]] = x[master[k]], k < n
void copy_images(int n, const int32_t* img, const int32_t* master, double* x, hipStream_t s);
// max |u_node| and max over cells of max(1e-10, max|u|)/diam -> out[0], out[1]
// (over the first n_cells cells of cd: the owned ones)
void velocity_stats(const CellData& cd, int n_cells, const double* u, double* out2, hipStream_t s);
// min/max of a vector -> out[0] = min, out[1] = max
void minmax(int n, const double* x, double* out2, hipStream_t s);
// block of a CSR matrix: rows [r0, r1), columns [c0, c1) (other columns skipped):
// y[r - r0] (+)= sum_k val[k] x[col[k] - c0]
void spmv_block(int r0, int r1, int c0, int c1, const int32_t* ptr, const int32_t* col,
                const double* val, const double* x, double* y, bool add, hipStream_t s);
void shift(int n, DScal c, double* y, hipStream_t s);                         // y += c
void zero_fixed(int n, const uint8_t* fixed, double* y, hipStream_t s);       // y[fixed] = 0
// halo staging: buf[k] = v[pos[k]] / v[pos[k]] = buf[k], k < n
void gather(int n, const int32_t* pos, const double* v, double* buf, hipStream_t s);
void scatter(int n, const int32_t* pos, const double* buf, double* v, hipStream_t s);

}  // namespace dcp
