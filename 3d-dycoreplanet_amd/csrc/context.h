// Device-resident state of one dcp_ctx (one GPU / rank).
#pragma once
#include <chrono>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include <memory>
#include <mutex>
#include <thread>
#include <utility>

#include "../../include/dcp.h"
#include "comm.h"
#include "device.h"
#include "feec.h"

namespace dcp {

// a failed C-ABI call: its return code and message (dcp_last_error)
struct ApiError {
  int code;
  std::string msg;
};

// Device bytes held by the buffers each host thread allocated (one rank = one
// thread in an in-process group): dcp_device_memory reports the calling
// thread's. One process-wide table behind a mutex, each buffer remembering its
// allocating thread, so a buffer freed on another thread (e.g. a context closed
// by Python's GC) is still taken off its owner's count.
struct DevMemTrack {
  int64_t live = 0, peak = 0;
};
struct DevMemTable {
  std::mutex mu;
  std::unordered_map<std::thread::id, DevMemTrack> per_thread;
  std::unordered_map<const void*, std::pair<int64_t, std::thread::id>> sizes;
};
inline DevMemTable& dev_mem_table() {
  static DevMemTable* t = new DevMemTable;  // never destroyed: frees may run during exit
  return *t;
}
inline DevMemTrack dev_mem() {
  DevMemTable& t = dev_mem_table();
  std::lock_guard<std::mutex> lock(t.mu);
  auto it = t.per_thread.find(std::this_thread::get_id());
  return it == t.per_thread.end() ? DevMemTrack{} : it->second;
}
inline void dev_mem_alloc(const void* p, size_t bytes) {
  DevMemTable& t = dev_mem_table();
  const auto me = std::this_thread::get_id();
  std::lock_guard<std::mutex> lock(t.mu);
  auto old = t.sizes.find(p);
  if (old != t.sizes.end()) t.per_thread[old->second.second].live -= old->second.first;
  t.sizes[p] = {int64_t(bytes), me};
  DevMemTrack& m = t.per_thread[me];
  m.live += int64_t(bytes);
  if (m.live > m.peak) m.peak = m.live;
}
inline void dev_mem_free(const void* p) {
  DevMemTable& t = dev_mem_table();
  std::lock_guard<std::mutex> lock(t.mu);
  auto it = t.sizes.find(p);
  if (it == t.sizes.end()) return;
  t.per_thread[it->second.second].live -= it->second.first;
  t.sizes.erase(it);
}

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  ~DBuf() { release(); }
  void release() {
    if (p) {
      dev_mem_free(p);
      (void)hipFree(p);
    }
    p = nullptr;
    n = 0;
  }
  void alloc(size_t count) {
    release();
    if (count == 0) count = 1;
    DCP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
    dev_mem_alloc(p, count * sizeof(T));
    n = count;
  }
  void upload(const std::vector<T>& h) {
    alloc(h.size());
    if (!h.empty()) DCP_HIP_CHECK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  }
  void zero(hipStream_t s) { DCP_HIP_CHECK(hipMemsetAsync(p, 0, n * sizeof(T), s)); }
};

struct Timer {
  hipEvent_t a = nullptr, b = nullptr;
  int count = 1;  // operator applies between a and b (averages divide by it)
  void init() {
    DCP_HIP_CHECK(hipEventCreate(&a));
    DCP_HIP_CHECK(hipEventCreate(&b));
  }
  void destroy() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    a = b = nullptr;
  }
};

struct Ctx {
  // SolverControl log of one solve (log_history / log_result): every
  // check(step, value) and the result (0 iterating, 1 convergence, 2 failure)
  struct SolverLog {
    std::vector<std::pair<unsigned, double>> checks;
    int result = 0;
  };
  SolverLog solver_log[2];           // the FGMRES attempts of the last dcp_solve_nse
  bool log_history = false;          // DCP_OPT_LOG_HISTORY
  // TimerOutput of the reference (computing_timer): wall time and calls per
  // section, in first-use order, under the reference's section names
  struct Section {
    std::string name;
    long calls = 0;
    double seconds = 0;
  };
  std::vector<Section> sections;
  std::chrono::steady_clock::time_point t_created = std::chrono::steady_clock::now();
  void section_add(const char* name, double s) {
    for (auto& x : sections)
      if (x.name == name) {
        ++x.calls;
        x.seconds += s;
        return;
      }
    sections.push_back(Section{name, 1, s});
  }
  dcp_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  dcp_physics hph{};
  PhysicsDev ph{};
  bool have_physics = false, have_mesh = false;

  // local sizes (owned + ghost on several GPUs; the whole mesh on one)
  int n_cells = 0, n_u = 0, n_p = 0, n_T = 0, n_vnodes = 0;
  // owned parts (rows this rank computes) and global sizes
  int n_owned_cells = 0, nvo = 0, npo = 0, nTo = 0;
  int n_u_g = 0, n_p_g = 0, n_T_g = 0;
  // multi-GPU: communicator (null on one GPU), halo plans, local->global maps
  std::unique_ptr<Comm> comm;
  struct Halo {
    std::vector<int> peers;
    std::vector<size_t> sn, rn, soff, roff;
    int ns = 0, nr = 0;
    DBuf<int32_t> spos, rpos;    // positions in the vector (send: owned, recv: ghost)
    DBuf<double> sbuf, rbuf;
  };
  Halo halo_v, halo_p, halo_nse, halo_T;
  std::vector<int32_t> vnode_g, p_g, T_g;
  // max over ranks of |seg_nse|, |seg_p|, |seg_v|, |seg_T|, FEEC |[w u p]|, |w|, |u|, |p|
  int max_owned[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int sell_part_len = 0;             // common length of the SELL partial arrays
  // mesh
  DBuf<int32_t> cell_q2, cell_p, cell_T;
  int tdpc3 = 8;                      // temperature dofs per 3D cell: 8 (FE_Q(1)) or 27 (FE_Q(2))
  DBuf<double> cell_geo, diameter, T_bc;
  DBuf<NodeConstraint> vcon;
  DBuf<uint8_t> T_fixed;
  std::vector<int> color_ptr;  // cells of colour k: color_cells[color_ptr[k] .. color_ptr[k+1])
  DBuf<int32_t> color_cells;
  // block-CSR patterns + values
  DBuf<int32_t> A_ptr, A_col, Bt_ptr, Bt_col, B_ptr, B_col, T_ptr, T_col;
  DBuf<double> A_val, Bt_val, B_val, Tmass, Tstiff, Tmat;
  size_t A_nnzb = 0;                 // blocks of the A pattern (A_val allocated on first use)
  DBuf<int32_t> posA, posBt, posB, posT;
  // scatter positions carry first-touch marks (no zero fill before assembly)
  bool first_touch_A = false, first_touch_Bt = false, first_touch_B = false;
  // B^T by tasks of rows on the separable shell (assembly.hip k_bt_tasks):
  // task headers and (row, cell) slot records [4 int32 each], built at upload
  bool bt_rows = false;
  DBuf<int32_t> bt_task_hdr, bt_slot_rec;
  int bt_ntasks = 0;
  int bt_slots = 16;  // slot records per task (8 or 16)
  // several GPUs: per colour the cells with an owned velocity node (the rhs)
  std::vector<int> rhs_color_ptr;
  DBuf<int32_t> rhs_color_cells;
  // the rhs in cell order (mf_rhs_cells + gather, DCP_ASM_RHS_CELL_ORDER=0 off):
  // per colour the cells with a constrained node, for the constrained diagonals
  bool rhs_cell_order = false;
  std::vector<int> con_color_ptr;
  DBuf<int32_t> con_color_cells;
  DBuf<int32_t> con_cptr, con_cslot;  // slots of the constrained diagonals (con_gather)
  DBuf<double> con_cbuf;
  // the same diagonals in Kronecker form (k_cdk_*, one GPU, layered shell):
  // per slot its (lateral, radial) table indices, per node its constrained
  // components, and the lateral / radial tables
  bool cdk = false;
  DBuf<int32_t> cdk_rec, cdk_mask;
  DBuf<double> cdk_L, cdk_R;
  DBuf<double> bt_P;  // [n_cols][216] column factors, then [n_layers][12] layer factors (upload)
  double* bt_Q = nullptr;
  int bt_ncols = 0;
  // blocks some cell's scatter position reaches (first-touch marking at upload)
  unsigned long long touched_A = 0, touched_Bt = 0, touched_B = 0;
  // nse_matrix in operator form: B^T, B and the diagonal of the constrained
  // velocity rows (con_diag, [constrained node][3], indexed by mf_cidx) are
  // assembled; the velocity-velocity block A is applied matrix-free and
  // materialised into A_val only when read (export, DCP_OPT_MATRIX_FREE = 0)
  // or when DCP_OPT_ASSEMBLE_VELOCITY_BLOCK asks for it on every assembly.
  DBuf<double> con_diag;            // [3 n_con | n_pimg]: velocity nodes, then pressure images
  int n_con = 0;
  // periodic identification (HostPrep): original cell maps, image lists
  // (dof, partner) per field for distribute, pressure image index, the A
  // pattern position of each velocity image's diagonal block, and the T
  // pattern position of each image's own diagonal per cell vertex
  DBuf<int32_t> cell_q2o, cell_po, cell_To, pcidx, posTs;
  DBuf<int32_t> img_u, mst_u, img_p, mst_p, img_T, mst_T, img_node;
  DBuf<int64_t> img_blk;
  int n_img_u = 0, n_img_p = 0, n_img_T = 0, n_img_node = 0;
  bool periodic = false;
  bool assemble_A = false;   // DCP_OPT_ASSEMBLE_VELOCITY_BLOCK
  bool element_mfma = false;  // DCP_OPT_ELEMENT_MFMA
  // B entry k = B^T entry B_tperm[k] (every B entry has its B^T partner, one
  // GPU): the operator form scatters B^T only and copies B from it
  DBuf<int32_t> B_tperm;
  bool B_transpose = false;
  // Schur-complement solver: ILU(0) structure of the velocity block (built on
  // first use) and its factor
  struct Ilu {
    DBuf<int32_t> ptr, col, diag, pos, lf_ptr, lf_rows, lb_ptr, lb_rows, p_img;
    std::vector<int> lf_host;
    DBuf<double> lu;
    int n = 0, n_lf = 0, n_lb = 0, n_p_img = 0, max_row = 0;
    // forget the structure and the factor (a new mesh may have the same n_u
    // with another numbering or pattern)
    void reset() {
      for (auto* b : {&ptr, &col, &diag, &pos, &lf_ptr, &lf_rows, &lb_ptr, &lb_rows, &p_img})
        b->release();
      lu.release();
      lf_host.clear();
      n = n_lf = n_lb = n_p_img = max_row = 0;
    }
    IluView view() const {
      return IluView{n,         long(col.n), ptr.p,     col.p,      diag.p,    pos.p,
                     n_lf,      n_lb,        lf_ptr.p,  lf_rows.p,  lb_ptr.p,  lb_rows.p};
    }
  } ilu;
  std::vector<double*> sc_v, sc_p;  // Schur-complement solver work vectors (velocity / pressure)
  bool B_current = true;     // B_val holds the B block of the last assembly
  bool A_current = false;    // A_val holds the block of the last assembly
  PhysicsDev nse_ph{};       // physics (dt) of the last assemble_nse_system
  // explicit Schur complement S = B D_A^-1 B^T (CSR over pressure dofs)
  DBuf<int32_t> S_ptr, S_col;
  // its values live in the SELL-64 layout of that pattern (sell_spmv)
  DBuf<int64_t> S_sell_off;
  DBuf<int32_t> S_sell_col;          // 32-bit columns, or
  DBuf<uint16_t> S_sell_c16;         // 16-bit offsets from S_sell_base[slice]
  DBuf<int32_t> S_sell_base;
  DBuf<int32_t> S_pmap;              // CSR entry of S -> SELL position
  DBuf<int32_t> S_perm;              // SELL row r = pressure dof S_perm[r] (null: identity)
  DBuf<double> sperm_x, sperm_b;     // permuted-order work vectors
  // structured columns (SellView::nbr): lateral neighbour table [j][nc]
  DBuf<int32_t> S_nbr;
  int S_nc = 0, S_nl = 0, S_nj = 0;
  SellView sell() const {
    SellView v{npo, S_sell_off.p, S_sell_col.p, S_sell_c16.p, S_sell_base.p, S_val.p};
    if (S_nbr.p) {
      v.nbr = S_nbr.p;
      v.nc = S_nc;
      v.nl = S_nl;
      v.nj = S_nj;
    }
    return v;
  }
  DBuf<double> S_val;
  long S_version = 0;                // formations of S_val (matrix powers: ghost values current?)
  // several GPUs, s-step inner solve: matrix powers (matpow.cpp). Ghost rows
  // of S (depth 1..3 from the owned rows, by depth) in SELL-64 with a row map
  // into the extended pressure vector [local dofs | further dofs the ghost
  // rows reach], their values from the owners, and the depth-4 halo
  bool matrix_powers = true;         // DCP_OPT_MATRIX_POWERS
  struct MatPow {
    bool built = false;
    int n_ext = 0;                   // extended pressure vector length
    int rows[4] = {0, 0, 0, 0};      // ghost rows of depth <= 0, 1, 2, 3
    DBuf<int64_t> off;
    DBuf<int32_t> col, rowmap;
    DBuf<double> val;
    Halo halo;                       // depth-4 halo of a block's start vector
    Halo vals;                       // owner SELL positions -> ghost SELL positions
    long version = -1;               // the S_version of val
    SellView view(int depth) const {
      return SellView{rows[depth], off.p, col.p, nullptr, nullptr, val.p, rowmap.p};
    }
    void reset();
  } mp;
  DBuf<double> sell_part;            // 2 x sell_fused_blocks(n_p) partials
  int S_max_row = 0;
  bool schur_explicit = true;
  // matrix-free operator (kernels/matfree.hip): geometry, first-touch bits,
  // constrained velocity dofs with their assembled diagonal entries
  // 0: assembled block-CSR; 1 (default): cell-order pencil kernel + node
  // gather (MfCells / MfGather); 2: colour-class launches (MfData)
  int matrix_free = 1;
  DBuf<double> mf_geo;                  // colour order (see MfData)
  DBuf<double> mf_geo_tree;             // tree order, non-separable meshes (MfCells::geo)
  DBuf<int32_t> mf_q2, mf_p;
  DBuf<uint64_t> mf_first;
  DBuf<int32_t> mf_cdof;
  DBuf<int64_t> mf_cpos;
  int mf_ncon = 0, mf_ncon_v = 0;  // fix-up entries: all / velocity dofs only
  DBuf<double> mf_buf;  // dof-sorted partial sums (velocity: one per node and cell group)
  DBuf<uint32_t> mf_cmask;
  DBuf<int32_t> mf_vptr, mf_pptr, mf_vslot, mf_pslot, mf_cidx, mf_vorder, mf_porder;
  DBuf<MfLink> mf_vnext;
  DBuf<uint8_t> mf_wcon;
  int32_t mf_pbase = 0;
  // chunked apply (DCP_MF_CHUNKS > 1 at upload): the gather of chunk k's
  // finished dofs runs on mf_stream while the pencil kernel works chunk k + 1.
  // Measured slower at r=5 (the pencil launch fills every CU's LDS, so the
  // gather cannot co-reside; each extra launch + event pair costs ~5 us):
  // default 1 = both launches on the context stream.
  static constexpr int kMfChunksMax = 16;
  int mf_chunks = 1;
  std::vector<int> mf_cell_cut, mf_vcut, mf_pcut;  // [mf_chunks + 1] each
  hipStream_t mf_stream = nullptr;
  hipEvent_t mf_chunk_ev[kMfChunksMax] = {}, mf_join_ev = nullptr;
  DBuf<int32_t> mf_col, mf_layer;
  DBuf<double> mf_colgeo, mf_laygeo, mf_colphi, mf_layR, mf_colphin, mf_layRs;
  bool mf_separable = false;
  // the fused one-launch apply (k_mf_fused, DCP_MF_FUSED): schedule, gather
  // window dependencies, per-batch done flags, the apply counter (flag tags)
  DBuf<int32_t> mf_sched, mf_dep_ptr, mf_dep;
  DBuf<uint32_t> mf_done;
  int mf_ntasks = 0, mf_nvwin = 0;
  unsigned mf_seq = 0;
  bool mf_fused = false;
  MfFused mff(double* err) const {
    return MfFused{mf_sched.p, mf_dep_ptr.p, mf_dep.p, const_cast<uint32_t*>(mf_done.p), err,
                   mf_nvwin, 1L << 22};
  }
  MfCells mfc() const {
    return MfCells{n_cells,    n_u,         cell_q2.p,  cell_p.p,
                   mf_geo_tree.p, vcon.p,   mf_cmask.p, mf_vslot.p, mf_vnext.p,
                   mf_pslot.p, mf_separable ? mf_col.p : nullptr,
                   mf_colgeo.p, mf_layer.p, mf_laygeo.p, cell_T.p, mf_colphi.p, mf_layR.p,
                   mf_colphin.p, mf_layRs.p};
  }
  MfGather mfg() const {
    // one chunk: the gather order is the identity (no order arrays read)
    return MfGather{n_vnodes,  n_p,      n_u,       mf_chunks > 1 ? mf_vorder.p : nullptr,
                    mf_chunks > 1 ? mf_porder.p : nullptr,
                    mf_vptr.p, mf_pptr.p, mf_pbase, mf_cidx.p,   vcon.p,
                    con_diag.p, periodic ? pcidx.p : nullptr, con_diag.p + 3 * size_t(n_con),
                    mf_wcon.p};
  }
  MfData mfd() const {
    return MfData{n_u, mf_q2.p, mf_p.p, vcon.p, mf_geo.p, mf_first.p};
  }
  // separable temperature assembly (tsep.cpp, kernels/temperature_sep.hip): set at upload
  // when the local cells are the full column x layer product of a separable
  // shell with FE_Q(1) temperature and no periodic identification
  bool tsep = false;
  int ts_n_colids = 0, ts_n_layers = 0, ts_n_kinds = 0, ts_n_latnnz = 0, ts_n_con = 0;
  DBuf<int32_t> ts_ord2lay, ts_lay2ord, ts_kind, ts_lptr, ts_lcon, ts_sptr, ts_slot;
  DBuf<uint16_t> ts_cmask;
  DBuf<uint32_t> ts_code, ts_rcode;
  DBuf<int32_t> ts_blk_ptr, ts_blk_rec;
  int ts_blk_pt = 0, ts_max_rec = 0;
  DBuf<double> ts_loc, ts_rad, ts_A, ts_rec;
  bool ts_tmat_valid = false;  // Tmat / T_inv of the last matrix assembly, made with ts_tmat_dt
  double ts_tmat_dt = 0.0;
  TSepDev tsd() const {
    TSepDev t;
    t.n_colids = ts_n_colids;
    t.n_layers = ts_n_layers;
    t.n_kinds = ts_n_kinds;
    t.n_latnnz = ts_n_latnnz;
    t.colgeo = mf_colgeo.p;
    t.laygeo = mf_laygeo.p;
    t.layR = mf_layR.p;
    t.ord2lay = ts_ord2lay.p;
    t.lay2ord = ts_lay2ord.p;
    t.kind = ts_kind.p;
    t.n_con = ts_n_con;
    const char* pr = std::getenv("DCP_TSEP_PROBE");
    t.probe = pr ? std::atoi(pr) : 0;
    t.cmask = ts_cmask.p;
    t.lptr = ts_lptr.p;
    t.lcon = ts_lcon.p;
    t.code = ts_code.p;
    t.blk_pt = ts_blk_pt;
    t.max_rec = ts_max_rec;
    t.blk_ptr = ts_blk_ptr.p;
    t.blk_rec = ts_blk_rec.p;
    t.rcode = ts_rcode.p;
    t.T_col = T_col.p;
    t.sptr = ts_sptr.p;
    t.slot = ts_slot.p;
    t.loc = ts_loc.p;
    t.rad = ts_rad.p;
    t.A = ts_A.p;
    t.rec = ts_rec.p;
    return t;
  }
  // B^T in Kronecker form (btkron.cpp, kernels/bt_kron.hip): set at upload on
  // the one-GPU layered shell; then every assembly (operator form or full)
  // takes B^T from it and B as its transpose
  bool btk = false;
  int btk_n_layers = 0, btk_n_kinds = 0, btk_n_pairs = 0, btk_n_con = 0, btk_n_conent = 0;
  int btk_max_rec = 0;
  DBuf<int32_t> btk_ord2lay, btk_kind, btk_lptr, btk_lcon, btk_blk_cptr, btk_blk_crow;
  int btk_max_con = 0;
  DBuf<int32_t> btk_blk_ptr, btk_blk_rec;
  DBuf<uint32_t> btk_code;
  DBuf<double> btk_A;
  BtkDev btkd() const {
    BtkDev b;
    b.n_layers = btk_n_layers;
    b.n_kinds = btk_n_kinds;
    b.n_pairs = btk_n_pairs;
    b.n_con = btk_n_con;
    b.n_conent = btk_n_conent;
    b.max_rec = btk_max_rec;
    b.P = bt_P.p;
    b.Q = bt_Q;
    b.ord2lay = btk_ord2lay.p;
    b.kind = btk_kind.p;
    b.lptr = btk_lptr.p;
    b.lcon = btk_lcon.p;
    b.code = btk_code.p;
    b.blk_ptr = btk_blk_ptr.p;
    b.blk_rec = btk_blk_rec.p;
    b.blk_cptr = btk_blk_cptr.p;
    b.blk_crow = btk_blk_crow.p;
    b.max_con = btk_max_con;
    b.A = btk_A.p;
    return b;
  }
  // state
  DBuf<double> nse_sol, old_nse, T_sol, old_T, nse_rhs, T_rhs;
  DBuf<double> A_diag, Mp_diag, A_inv, Mp_inv, T_inv;
  // scratch: reduction partials, device scalars
  DBuf<double> partials, dscal;
  double* hpinned = nullptr;   // pinned host mirror of small readbacks
  double* hmapped = nullptr;   // coherent mapped host memory: the chain timeout flag (one GPU)
  // one-launch Gram-Schmidt chains (k_mgs_chain): hand-off granules, launch
  // counter (the granule tags), CU count (residency bound), DCP_OPT_FUSED_CHAIN
  DBuf<double> chain_gran;
  unsigned long long chain_seq = 0;
  int n_cus = 0;
  bool fused_chain = true;
  int handoff_timeouts = 0;  // one-launch hand-offs that timed out (fused_chain then off)
  DBuf<double> inner_x0;     // the inner Schur solve's initial guess (rerun after a timeout)
  // DCP_OPT_GRAM_SCHMIDT: 0 = modified (deal.II SolverGMRES, default), 1 = the
  // inner Schur GMRES with classical Gram-Schmidt twice, 2 = DCGS2 (one
  // reduction per step), each restart cycle device-resident
  // (kernels/krylov.hip): state, polled status, partials, basis pointer table
  int gram_schmidt = 0;
  double S_lambda = 0;                // Gershgorin bound of S (s-step shifts), 0 = not yet formed
  DBuf<double> ss_c;                 // s-step block sums (several GPUs / large meshes)
  DBuf<double> head_part;  // per-slice |p|^2 partials of the fused restart head
  DBuf<GmresDev> gm_state;
  GmresReport* gm_report = nullptr;  // pinned [2]: the reports of the last two cycles
  hipEvent_t gm_ev[2] = {nullptr, nullptr};
  DBuf<double> gm_part;
  DBuf<double> dcgs_gran;            // hand-off granules of the DCGS2 steps (their own tag scheme)
  DBuf<unsigned> gm_cnt;             // last-block counter of the CGS2 launches
  DBuf<const double*> gm_ptrs;
  std::vector<const double*> gm_ptrs_host;
  int fgmres_max_outer = 40;         // SolverControl(40) of the first FGMRES (test hook)
  int inner_max_steps = 5000;        // SolverControl(5000) of the inner Schur GMRES (probe hook)
  int schur_fixed_inner = 0;         // DCP_OPT_SCHUR_FIXED_INNER (parity hook of solve_nse_schur)
  int block_fixed_inner = 0;         // DCP_OPT_BLOCK_FIXED_INNER (parity hook of block_prec)
  long a_solve_its = 0;              // AztecOO A-GMRES iterations of the last solve_nse
  // test hook, read at context creation: DCP_TEST_FORCE_REORTH_AT=k makes the
  // loss-of-orthogonality test at inner step k (a multiple of 5 minus 1) trigger
  int test_force_reorth_at = -1;
  bool nse_assembled = false, precond_built = false, T_matrix_ok = false, T_rhs_ok = false;
  // Krylov workspaces (lazily sized)
  std::vector<double*> fg_v, fg_z;   // FGMRES basis
  DBuf<double> fg_aux;
  std::vector<double*> sg_v;         // inner Schur GMRES basis (n_p, or mp.n_ext)
  size_t sg_len = 0;                 // length of the sg_v vectors
  DBuf<double> schur_tmp1, schur_tmp2, utmp;
  std::vector<double*> ag_v;         // fallback A-GMRES basis (n_u)
  DBuf<double> cg_g, cg_d, cg_h;
  DBuf<double> coef;                 // multi_axpy coefficients
  DBuf<const double*> ptrs;          // multi_axpy pointer table
  dcp_timings timings{};
  Timer ev_total;
  // sampled, deferred timing of Schur-complement applies (no host sync in the loop)
  static constexpr int kSchurEvents = 256, kSchurSampleEvery = 8;
  std::vector<Timer> schur_ev;
  int schur_ev_used = 0;
  long schur_calls = 0;
  bool time_schur = false;
  // several GPUs: the ghost entries of old_nse / old_T are current (set where
  // the library itself made them so: set_state, copy_state and advance_state
  // into an old field, which exchange them as the reference's ghosted
  // assignment old = new does; cleared by every other access to the field),
  // so assemble_nse_system need not exchange them again
  bool old_nse_ghosted = false, old_T_ghosted = false;
  bool old_external = false;  // a caller holds a device pointer to an old field
  // the same for the matrix-free applies: [0] Stokes, [1] velocity block
  static constexpr int kMfEvents = 128;
  std::vector<Timer> mf_ev[2];
  int mf_ev_used[2] = {0, 0};
  long mf_calls[2] = {0, 0};

  // ---- FEEC variant (config 4): n_u = n_w + n_u(faces), n_p = cells
  bool feec = false;
  bool feec_zero_mean = true;          // parameters.correct_pressure_to_zero_mean
  int feec_fixed_inner = 0;            // DCP_OPT_FEEC_FIXED_INNER (test hook)
  int fe_nw = 0, fe_nu = 0, fe_np = 0;             // local (owned + ghost)
  int fe_nwo = 0, fe_nuo = 0, fe_npo = 0;          // owned
  int fe_nw_g = 0, fe_nu_g = 0;                    // global
  std::vector<int32_t> fe_w_g, fe_u_g;             // local -> global (several GPUs)
  Halo halo_fw, halo_fu, halo_fp;                  // per-field halos of [w | u | p] blocks
  // owned segments: the [w | u | p] vector and its blocks
  Seg seg_fe() const {
    return Seg{fe_nwo, fe_nw, fe_nwo + fe_nuo, fe_nw + fe_nu, fe_nwo + fe_nuo + fe_npo, 4};
  }
  Seg seg_fw() const { return Seg::all(fe_nwo, 5); }
  Seg seg_fu() const { return Seg::all(fe_nuo, 6); }
  Seg seg_fp() const { return Seg::all(fe_npo, 7); }
  DBuf<int32_t> fe_dofs;
  DBuf<int8_t> fe_sign;
  DBuf<double> fe_X, fe_cellw;
  DBuf<double> fe_cellw2;  // QGauss(2) cell volumes (PreconditionerBlockIdentity's mean)
  DBuf<uint8_t> fe_fixed;
  DBuf<int32_t> fe_ptr, fe_col, fe_pos, fp_ptr, fp_col, fp_pos;
  DBuf<double> fe_val, fp_val, fe_dinv;   // system, preconditioner, Jacobi of the w/u diagonal blocks
  double fe_wsum = 0;                      // sum of the mean-value weights
  double fe_wsum2 = 0;
  bool feec_block_prec = true;  // use_block_preconditioner_feec
  int T_fixed_cg = 0;            // DCP_OPT_T_FIXED_CG (test hook of solve_temperature)
  bool fe_assembled = false, fe_precond = false;
  std::vector<double*> fe_v, fe_s, fe_n;  // Krylov bases: outer, shifted Schur, nested Schur
  DBuf<double> fe_t1, fe_t2, fe_t3, fe_t4;
  FeecCellData fcd() const {
    return FeecCellData{n_cells, fe_dofs.p, fe_sign.p, fe_X.p, diameter.p, fe_fixed.p, cell_T.p};
  }

  // ---- two-dimensional model (Standard::BoussinesqModel<2>, dcp_mesh2d_upload):
  // nse_matrix [u | p] as one scalar CSR, blocks applied as row/column windows
  bool dim2 = false;
  int vdim = 3;                          // velocity components per support point
  int m2_tdpc = 4;                       // temperature dofs per cell (FE_Q(1) / FE_Q(2))
  DBuf<int32_t> m2_dofs, m2_tdofs, m2_pos, m2_posT;
  DBuf<double> m2_X, m2_srcw;
  DBuf<int8_t> m2_src;
  DBuf<uint8_t> m2_fixed;
  DBuf<int32_t> m2_ptr, m2_col;
  DBuf<double> m2_val;
  // NSE constraint lines (distribute) and the pressure dofs among them
  int m2_nlines = 0;
  DBuf<int32_t> m2_ldof, m2_lptr, m2_lent;
  DBuf<double> m2_lw, m2_linh;
  Mesh2DDev m2() const {
    return Mesh2DDev{n_cells, n_u,      m2_tdpc,    m2_dofs.p, m2_tdofs.p, m2_X.p,    diameter.p,
                     m2_src.p, m2_srcw.p, m2_fixed.p, m2_pos.p,  m2_posT.p,  T_fixed.p, T_bc.p};
  }
  // y = block (rows [r0, r1), columns [c0, c1)) of the 2D nse_matrix times x
  // (x indexed from c0)
  void m2_block(int r0, int r1, int c0, int c1, const double* x, double* y, bool add) const {
    spmv_block(r0, r1, c0, c1, m2_ptr.p, m2_col.p, m2_val.p, x, y, add, stream);
  }

  Seg seg_nse() const { return Seg::two(vdim * nvo, n_u, vdim * nvo + npo, 0); }
  Seg seg_p() const { return Seg::all(npo, 1); }
  Seg seg_v() const { return Seg::all(vdim * nvo, 2); }
  Seg seg_T() const { return Seg::all(nTo, 3); }

  CellData cd() const {
    CellData c;
    c.n_cells = n_cells;
    c.cell_q2 = cell_q2.p;
    c.cell_p = cell_p.p;
    c.cell_T = cell_T.p;
    c.tdpc = tdpc3;
    c.geo = cell_geo.p;
    c.vcon = vcon.p;
    c.T_fixed = T_fixed.p;
    c.T_bc = T_bc.p;
    c.diameter = diameter.p;
    c.cell_q2o = periodic ? cell_q2o.p : nullptr;
    c.cell_po = periodic ? cell_po.p : nullptr;
    c.cell_To = periodic ? cell_To.p : nullptr;
    const bool sep = mf_separable && mf_colphi.p != nullptr;
    c.sep_col = sep ? mf_col.p : nullptr;
    c.sep_colgeo = sep ? mf_colgeo.p : nullptr;
    c.sep_colphi = sep ? mf_colphi.p : nullptr;
    c.sep_layer = sep ? mf_layer.p : nullptr;
    c.sep_laygeo = sep ? mf_laygeo.p : nullptr;
    c.sep_layR = sep ? mf_layR.p : nullptr;
    return c;
  }
  ScatterMaps maps() const { return ScatterMaps{posA.p, posBt.p, posB.p, posT.p}; }
  int n_colors() const { return int(color_ptr.size()) - 1; }
  const int32_t* color_begin(int k) const { return color_cells.p + color_ptr[k]; }
  int color_size(int k) const { return color_ptr[k + 1] - color_ptr[k]; }
  ~Ctx();
};

// TimerOutput::Scope: wall time of the enclosed work (the stream is
// synchronised at the end of the scope) under a reference section name
struct SectionScope {
  Ctx& c;
  const char* name;
  std::chrono::steady_clock::time_point t0;
  bool done = false;
  SectionScope(Ctx& ctx, const char* n) : c(ctx), name(n), t0(std::chrono::steady_clock::now()) {}
  void stop() {
    if (done) return;
    done = true;
    (void)hipStreamSynchronize(c.stream);
    c.section_add(name, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  ~SectionScope() { stop(); }
};

// api.cpp: A_val allocated for the A pattern (if not yet)
void ensure_A_val(Ctx& c);
// api.cpp: A_val <- nse_matrix.block(0,0) of the last assembly (if not current)
void materialize_velocity_block(Ctx& c);
// B = (B^T)^T after an operator-form assembly that scattered B^T only
void materialize_B(Ctx& c);
// model2d.cpp: the 2D model's upload and hot-path members
void mesh2d_upload(Ctx& c, const dcp_mesh2d* m);
void mesh2d_check(const dcp_mesh2d* m, int* n_colors);
void assemble_nse_2d(Ctx& c, int flags);
void build_precond_2d(Ctx& c);
void assemble_T_matrix_2d(Ctx& c);
void assemble_T_rhs_2d(Ctx& c);
void distribute_nse_2d(Ctx& c, double* x);
void nse_matrix_export_2d(Ctx& c, int64_t* nnz, int32_t* rowptr, int32_t* cols, double* vals);
void cell_nse_system_2d(Ctx& c, int first, int n, double* K, double* f);
// tsep.cpp: the separable temperature tables (false: keep the colour kernels)
bool build_tsep(Ctx& c, int n_cells, const std::vector<int32_t>& td, const std::vector<int32_t>& col,
                const std::vector<int32_t>& layer, const std::vector<double>& layR,
                const std::vector<uint8_t>& Tfix, const std::vector<double>& Tbc,
                const std::vector<int32_t>& Tp,
                const std::vector<int32_t>& Tc, int n_T);
// btkron.cpp: the Kronecker B^T tables (false: keep the B^T tasks)
bool build_btk(Ctx& c, int n_cells, const std::vector<int32_t>& q2, const std::vector<int32_t>& pd,
               const std::vector<int32_t>& col, const std::vector<int32_t>& layer,
               const std::vector<double>& layR, const std::vector<NodeConstraint>& vc,
               const std::vector<int32_t>& Btp, const std::vector<int32_t>& Btc, int nv, int n_p);
// solver.cpp
int solve_nse(Ctx& c, int* outer, int* inner);
// solve_NSE_Schur_complement (boussinesq_model.tpp:1248-1414)
int solve_nse_schur(Ctx& c, int* schur_iterations, int* a_solves);
int solve_temperature(Ctx& c, int* iters, double* T_range);
void nse_vmult(Ctx& c, const double* src, double* dst);
// hmapped slot of the fused matrix-free apply's poll-timeout flag
constexpr int kMfErrSlot = 8001;
// a fused matrix-free apply whose gather poll timed out (k_mf_fused): throws
// and switches the context to the two-launch apply
void check_mf_err(Ctx& c);
void velocity_vmult(Ctx& c, const double* src, double* dst);
void schur_vmult(Ctx& c, const double* src_p, double* dst_p);
int block_preconditioner_vmult(Ctx& c, const double* src, double* dst, bool do_solve_A,
                               int* inner);
void free_workspaces(Ctx& c);
void ensure_workspaces(Ctx& c);
// FEEC solve (solve_NSE_block_preconditioned, boussineq_model_FEEC.tpp:1268-1477)
int feec_solve_nse(Ctx& c, int* iterations);
// multi-GPU plumbing (no-ops on one GPU)
int chain_width(const Ctx& c, Seg g);
void allreduce(Ctx& c, double* buf, size_t n, bool max = false);
void halo_exchange(Ctx& c, Ctx::Halo& h, double* v);
// matpow.cpp: build the matrix powers (collective, once per mesh) and copy the
// ghost rows' values from their owners when S was formed again (collective)
void matpow_setup(Ctx& c);
void matpow_prepare(Ctx& c);

}  // namespace dcp
