// Host side of the MI355X-native dycore: field registry in HBM, the atm_srk3
// sequencer (mpas_atm_time_integration.F:142-1796), halo exchanges between
// blocks (mpas_dmpar.F: device copies between blocks of this process, RCCL
// send/recv between processes) and the C ABI declared in include/mpas_dycore.h.
// One translation unit with the kernels.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>
#include <unistd.h>

// The library links two builds of this file (gen_api.py): MPAS_API_TAG=n, one wavefront per
// column (nVertLevels 4..63), and MPAS_API_TAG=w with MPAS_WIDE, one workgroup per column
// (64..127); each build's entry points are renamed, and api_dispatch.cpp routes the public ones.
#ifdef MPAS_API_TAG
#include "api_rename.h"
#endif
#include "../../include/mpas_dycore.h"
#include "kernels.hip"
#include "halo.hip"
#include "summary.hip"
#include "lbc.hip"
#include "model_init.hip"

using namespace mpas;

namespace {

enum Loc { L_CELL, L_EDGE, L_VERTEX, L_NONE };
enum Target { T_NONE, T_CELL, T_EDGE, T_VERTEX, T_SMALL };  // int index semantics

struct Field {
  std::string pool, name;
  Loc loc;
  int64_t inner;      // doubles/ints per element (Fortran leading dims product)
  bool is_int;
  Target target;
  int ntl;
  int nsub = 1;       // > 1: scalar-major [nsub][n+1][inner/nsub] in HBM, Fortran image (nsub, inner/nsub, n+1)
  void* buf[2] = {nullptr, nullptr};
  // buffer rotation of the step (srk3 rotate_saves / swap_theta): rot >= 0 names the partner field
  // (X <-> X_save) whose buffer this field trades at every rotation, rot_pos counts the trades mod 2
  // (which of the two buffers it holds); flip = the time levels of a state field are swapped
  int rot = -1, rot_pos = 0, flip = 0;
  // mesh fields strided by maxEdges (me = 1) or maxEdges2 (me = 2): buf holds the Fortran image at the
  // declared size (what set/get_field and the device pointer see), `packed` the same array at the
  // block's effective strides (pack_mesh), which is what the kernels read; nullptr: equal strides
  int me = 0;
  void* packed = nullptr;
  int64_t packed_inner = 0;
  // allocated at its first set_field: the inputs only the model-init precompute reads (deriv_two, zb,
  // zb3, meshDensity, areaCell, areaTriangle -- mpas_dyc_model_init)
  bool lazy = false;
};

// One entry of a block's multihalo exchange list (mpas_multihalo_exchange_list:
// procID, blockID, nList, srcList/destList), one per (location, halo layer,
// direction, peer block).
struct XList {
  int loc, layer, dir, peer_rank, peer_block;
  int n = 0;
  int* d_idx = nullptr;  // 0-based local element indices, message order
  std::vector<int32_t> h_idx;  // the same on the host (fused-pack maps)
  // a positional list (mpas_dyc_set_exchange_positions, peer_block -1): element i takes slot
  // d_pos[i] (0-based) of the (loc, layer) region of the message to / from rank peer_rank, whose
  // slots all blocks of this process fill together -- mpas_dmpar's per-task buffers
  int* d_pos = nullptr;
  std::vector<int32_t> h_pos;
};

// A block: MPAS block_type -- dims, fields and exchange lists of one patch.
struct Block {
  Dims d{};
  std::vector<Field> fields;
  std::map<std::string, int> by_name;  // "pool.name"
  std::vector<XList> xl;
  int64_t nEdges_act = -1;             // edges with an owned cell (from cellsOnEdge), for B_ac
  std::vector<int32_t> h_coe, h_eoc, h_noc;  // host copies (0-based) for the halo-boundary flags
  std::vector<int32_t> h_voe, h_eov;         // verticesOnEdge / edgesOnVertex (0-based): fused u unpack
  std::vector<int32_t> h_noe;                // nEdgesOnEdge (pack_mesh)
  // maxEdges / maxEdges2 as the host declared them (the mesh file's dimensions; Fortran images and
  // h_eoc use these strides).  d.maxEdges / d.maxEdges2 are the strides the kernels index with:
  // max(nEdgesOnCell) and the edgesOnEdge slots the kernels need after pack_mesh
  int me_decl = 0, me2_decl = 0;
  // summarize_timestep records (summary.hip): partials and one SUM_REC record per field
  double* sum_part = nullptr;
  double* sum_out = nullptr;
};

// One RCCL message of an exchange point: a contiguous range of the process-wide send or receive buffer.
struct XMsg {
  int block, peer_rank, peer_block;
  int64_t off, count;  // doubles
};

// An exchange point, compiled: `pre` packs RCCL messages and copies halos between blocks of
// this process directly (owned columns of one block -> halo columns of another); `post`
// unpacks received RCCL messages.  One kernel launch each, whatever the number of blocks.
struct XPlan {
  XSeg* d_pre = nullptr;
  XSeg* d_post = nullptr;
  int npre = 0, npost = 0, maxn_pre = 0, maxn_post = 0;
  double* sendbuf = nullptr;
  double* recvbuf = nullptr;
  std::vector<XMsg> rsend, rrecv;  // in matching order
  bool warmed = false;              // its RCCL group has run once outside graph capture (warm_rccl)
  // fused pack (the per-sub-step rtheta_pp [+ rho_pp] exchange with RCCL peers only): the
  // acoustic cell phase writes the send buffer itself, so exchange() launches no pack kernel
  bool fused_pack = false;
  std::vector<PackMap> pack;        // per block
  // fused unpack: the exchange launches no unpack kernel; its consumer (the next acoustic edge
  // phase or the stage's last damping) reads the receive buffer through `unpack`
  bool fused_unpack = false;
  std::vector<UnpackMap> unpack;    // per block
  std::vector<void*> pack_mem;      // device allocations behind `pack`
  // the 876-887 and 642 exchanges fused into their producers and consumers (XPack / XUnpack,
  // dycore.h): then
  // fused_pack and fused_unpack are set too and these hold the per-block maps
  int fused_rec = 0;  // 1: the 876-887 exchange, 2: the tend_u exchange (642)
  std::vector<XPack> rpk_cell, rpk_edge;
  std::vector<XUnpack> rup_cell, rup_edge;
  // one-sided transfer (mpas_dyc_ctx::p2p, halo.hip k_p2p_post / k_p2p_get): the send buffer is
  // device memory the peers map; p2p_id < 0 until p2p_setup has exchanged the mappings
  bool p2p = false;
  int p2p_id = -1;
  unsigned long long* p2p_cnt = nullptr;  // [0] use counter, [1 + i] chunks pulled from get peer i
  P2PGet* d_get = nullptr;
  int nget = 0, get_chunks = 0;
  unsigned long long** d_ready = nullptr;  // the ready flags this rank raises (one per receiving rank)
  int nready = 0;
  const unsigned long long** d_cons = nullptr;  // the consumed flags this rank waits for
  int ncons = 0;
  std::vector<void*> p2p_mapped;  // the peers' send buffers mapped here (IPC)
  // pull (k_p2p_pull): block-pair lists, blocking exchanges -- the receiver copies the peers' owned
  // columns from their fields; no buffers, no pack / unpack kernels, no fused pack / unpack
  bool pull = false;
  std::vector<XSeg> h_pre, h_post;        // the pack / unpack segments (host), in buffer order
  std::vector<const std::vector<int32_t>*> h_pre_idx;  // each pack segment's send list (host)
  std::vector<int64_t> h_pre_off, h_post_off;
  XSeg* d_local = nullptr;                // in-process block-to-block copies of a pull plan
  int nlocal = 0, maxn_local = 0;
  P2PSeg* d_pseg = nullptr;
  int2* d_chunk = nullptr;                // (segment, first column) per workgroup of k_p2p_pull
  int npseg = 0, nchunk = 0, npeer_work = 0;
  P2PPeer* d_peer = nullptr;
  std::vector<void*> pull_mem;            // device copies of the peers' send lists
};

// One field of an exchange point: mpas_dmpar_exch_halo_field(field[, haloLayers]).
struct XField {
  const char* pool;
  const char* name;
  int tl;            // time level for state fields (1/2), ignored otherwise
  unsigned layers;   // bit l-1 set = halo layer l exchanged
};
constexpr unsigned ALL_LAYERS = 0x7u;

}  // namespace

struct mpas_dyc_ctx {
  Config cf{};
  int index_qv = 0;
  int device = 0;
  bool host_only = false;               // MPAS_DYC_HOST_ONLY: planner only, no device state
  hipStream_t stream = nullptr;
  std::vector<Block> blk;
  int cur = 0;                          // time level 1 -> buf[cur], 2 -> buf[1-cur]
  std::string err;
  hipEvent_t ev[8] = {};
  bool use_graph = false;
  bool graph_ran = false;               // the last step replayed a captured graph
  // captured steps, by buffer layout (layout_sig: the time level and the buffers the step's
  // rotations move, srk3 rotate_saves / swap_theta), and the dt each was captured for
  std::map<std::string, hipGraphExec_t> graphs;
  std::map<std::string, double> graph_dt;
  // halo exchange
  int rank = 0, nranks = 1;
  ncclComm_t comm = nullptr;
  bool rccl_local = false;              // route block-to-block copies of this process through RCCL too
  // MPAS_DYCORE_LOOPBACK=1 (timing only, tools/rank_emulation.py --exchange): the block of one rank
  // of an N-way run, with its real lists to the other ranks, alone on one GPU; every message goes to
  // this rank itself over a one-rank communicator (the halo receives this rank's own send data)
  // (=2: each pair is a hipMemcpyAsync instead of RCCL, to separate RCCL's own cost)
  int loopback = 0;
  // MPAS_DYCORE_P2P=1: messages between ranks of one node are pulled over xGMI by the receiving
  // rank's kernel (halo.hip k_p2p_get) instead of RCCL groups; RCCL stays for the set-up all-gathers
  int p2p = 0;
  unsigned long long* p2p_flags = nullptr;          // this rank's flag arena (uncached): [id][rank][2]
  std::vector<unsigned long long*> p2p_peer_flags;  // by rank: the arenas of the peers, mapped here
  std::vector<void*> p2p_mapped;                    // IPC mappings of the peers' arenas
  int p2p_nr = 0;                                   // rank stride of the arena
  int p2p_next = 0;                                 // the next exchange point's id
  int* p2p_status = nullptr;                        // set by a wait that timed out (halo.hip)
  std::vector<XField> p2p_open;                     // a split-phase p2p exchange between post and get
  bool p2p_pending = false;
  bool p2p_merge = true;                            // MPAS_DYCORE_P2P_MERGE=0: post and get as two launches
  bool p2p_pull = true;                             // MPAS_DYCORE_P2P_PULL=0: buffers + k_p2p_exchange instead
  std::map<std::pair<int, uint64_t>, void*> p2p_fields;  // (rank, its field buffer) -> mapped here
  // MPAS_DYCORE_LATE_ISSUE=1: a split-phase exchange is enqueued on the exchange stream at its
  // exchange_wait, after the compute kernels it overlaps (the same dependencies; only the order in
  // which a captured graph's nodes are created changes)
  bool late_issue = false;
  // MPAS_DYCORE_OVERLAP_ALL=1: split the 642 and 876-887 exchanges even with nothing to overlap (A/B)
  bool overlap_all = false;
  std::vector<XField> late_fs;
  bool late_pending = false;
  bool fused_pack_enabled = true;       // MPAS_DYCORE_FUSED_PACK=0: pack kernel instead (A/B)
  bool plain_exchange = false;          // mpas_dyc_halo_exchange: no fused pack / unpack
  bool lbc = false;                     // config_apply_lbcs (mpas_dyc_set_lbc)
  bool planning = false;                // dry run: build exchange plans, launch nothing
  std::set<std::string> planned;        // layouts whose exchange plans exist (plan_all)
  std::map<std::string, XPlan> plans;
  std::vector<std::string>* record = nullptr;  // mpas_dyc_plan_exchanges: keys of the calls, in order
  // split-phase exchanges: packs, RCCL and unpacks run on the exchange stream while the
  // compute stream works on elements that read no halo data
  hipStream_t xstream = nullptr;
  hipEvent_t xfork = nullptr, xjoin = nullptr;
  int overlap = -1;                     // 1 on, 0 off, -1 auto: on when exchanges go through RCCL
  bool bnd_ready = false;
  int physics = 0;                      // MPAS_DYC_PHYSICS_* flags (mpas_dyc_set_physics)
  // summarize_timestep: MPAS_DYC_PRINT_* modes reduced at the end of every step (the namelist
  // default is config_print_global_minmax_vel = true, Registry.xml:339)
  int summary_flags = MPAS_DYC_PRINT_GLOBAL_MINMAX_VEL;
  int summary_tl = 0;                   // time level the records describe (0: none yet)
  bool tail_pending = false;            // MPAS_DYC_PHYSICS_MICROPHYSICS: a step ran, mpas_dyc_finish_step not yet
  // exchange profile (mpas_dyc_set_profile): eager steps with HIP events around the exposed part of
  // every exchange (a blocking exchange whole; a split-phase one from the compute stream reaching
  // the join to the join's completion) and around every RCCL group
  bool profile = false;
  bool in_async = false;                // exchange() issued by exchange_async (on the exchange stream)
  std::vector<hipEvent_t> prof_exposed, prof_rccl;  // pairs (start, end)
  hipEvent_t prof_step[2] = {};
  double prof_out[5] = {};              // mpas_dyc_get_profile
  // the exchange whose RCCL group was enqueued last (a watchdog's report when a group hangs)
  char last_key[256] = {0};
  double* sum_gather = nullptr;         // RCCL all-gather buffer of the per-rank records
  // mpas_dyc_comm_init_host: the host's all-gather instead of an RCCL communicator (one-sided transfer)
  mpas_dyc_allgather_fn host_allgather = nullptr;
  void* host_user = nullptr;
};

namespace {

#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                      \
      return MPAS_DYC_EHIP;                                                           \
    }                                                                                 \
  } while (0)

#define NCCLCHK(x)                                                                    \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    if (r_ != ncclSuccess) {                                                          \
      ctx->err = std::string(#x) + ": " + ncclGetErrorString(r_);                     \
      return MPAS_DYC_ECOMM;                                                          \
    }                                                                                 \
  } while (0)

#define CHK(x)                 \
  do {                         \
    int r__ = (x);             \
    if (r__) return r__;       \
  } while (0)

int64_t nloc(const Block& b, Loc l) {
  switch (l) {
    case L_CELL: return b.d.nCells + 1;
    case L_EDGE: return b.d.nEdges + 1;
    case L_VERTEX: return b.d.nVertices + 1;
    default: return 1;
  }
}

int64_t field_elems(const Block& b, const Field& f) { return nloc(b, f.loc) * f.inner; }
int64_t field_bytes(const Block& b, const Field& f) { return field_elems(b, f) * (f.is_int ? 4 : 8); }

bool is_host_0d(const Field& f) {
  return f.pool == "mesh" && (f.name == "cf1" || f.name == "cf2" || f.name == "cf3");
}

void add(Block& c, const char* pool, const char* name, Loc loc, int64_t inner, int ntl = 1, bool is_int = false,
         Target t = T_NONE) {
  Field f;
  f.pool = pool;
  f.name = name;
  f.loc = loc;
  f.inner = inner;
  f.is_int = is_int;
  f.target = t;
  f.ntl = ntl;
  c.by_name[f.pool + "." + f.name] = (int)c.fields.size();
  c.fields.push_back(f);
}
// The Registry.xml var_structs the dycore touches (same list the oracle harness builds).
void build_registry(Block& c) {
  const int K = c.d.K, ME = c.d.maxEdges, ME2 = c.d.maxEdges2, ns = c.d.ns;
  // mesh: connectivity
  add(c, "mesh", "nEdgesOnCell", L_CELL, 1, 1, true);
  add(c, "mesh", "edgesOnCell", L_CELL, ME, 1, true, T_EDGE);
  add(c, "mesh", "cellsOnCell", L_CELL, ME, 1, true, T_CELL);
  add(c, "mesh", "verticesOnCell", L_CELL, ME, 1, true, T_VERTEX);
  add(c, "mesh", "kiteForCell", L_CELL, ME, 1, true, T_SMALL);
  add(c, "mesh", "cellsOnEdge", L_EDGE, 2, 1, true, T_CELL);
  add(c, "mesh", "verticesOnEdge", L_EDGE, 2, 1, true, T_VERTEX);
  add(c, "mesh", "nEdgesOnEdge", L_EDGE, 1, 1, true);
  add(c, "mesh", "edgesOnEdge", L_EDGE, ME2, 1, true, T_EDGE);
  add(c, "mesh", "nAdvCellsForEdge", L_EDGE, 1, 1, true);
  add(c, "mesh", "advCellsForEdge", L_EDGE, 15, 1, true, T_CELL);
  add(c, "mesh", "cellsOnVertex", L_VERTEX, 3, 1, true, T_CELL);
  add(c, "mesh", "edgesOnVertex", L_VERTEX, 3, 1, true, T_EDGE);
  // mesh: geometry
  for (const char* n : {"dcEdge", "dvEdge", "invDcEdge", "invDvEdge", "fEdge", "meshScalingDel2",
                        "meshScalingDel4", "specZoneMaskEdge", "angleEdge", "latEdge", "lonEdge"})
    add(c, "mesh", n, L_EDGE, 1);
  for (const char* n : {"invAreaCell", "specZoneMaskCell", "latCell", "lonCell"}) add(c, "mesh", n, L_CELL, 1);
  // regional LBCs (lbc.hip): zone masks, nearest relaxation cell, relaxation-zone mesh scaling
  add(c, "mesh", "bdyMaskCell", L_CELL, 1, 1, true);
  add(c, "mesh", "bdyMaskEdge", L_EDGE, 1, 1, true);
  add(c, "mesh", "nearestRelaxationCell", L_CELL, 1, 1, true, T_CELL);
  add(c, "mesh", "meshScalingRegionalCell", L_CELL, 1);
  add(c, "mesh", "meshScalingRegionalEdge", L_EDGE, 1);
  add(c, "mesh", "coeffs_reconstruct", L_CELL, 3 * (int64_t)ME);
  for (const char* n : {"invAreaTriangle", "fVertex"}) add(c, "mesh", n, L_VERTEX, 1);
  for (const char* n : {"fzm", "fzp", "rdzw", "rdzu", "u_init", "v_init"}) add(c, "mesh", n, L_NONE, K);
  for (const char* n : {"cf1", "cf2", "cf3"}) add(c, "mesh", n, L_NONE, 1);
  add(c, "mesh", "edgesOnCell_sign", L_CELL, ME);
  add(c, "mesh", "edgesOnVertex_sign", L_VERTEX, 3);
  add(c, "mesh", "kiteAreasOnVertex", L_VERTEX, 3);
  add(c, "mesh", "weightsOnEdge", L_EDGE, ME2);
  add(c, "mesh", "adv_coefs", L_EDGE, 15);
  add(c, "mesh", "adv_coefs_3rd", L_EDGE, 15);
  add(c, "mesh", "defc_a", L_CELL, ME);
  add(c, "mesh", "defc_b", L_CELL, ME);
  add(c, "mesh", "zgrid", L_CELL, K + 1);
  add(c, "mesh", "zz", L_CELL, K);
  add(c, "mesh", "zxu", L_EDGE, K);
  add(c, "mesh", "dss", L_CELL, K);
  add(c, "mesh", "t_init", L_CELL, K);
  add(c, "mesh", "zb_cell", L_CELL, (int64_t)ME * (K + 1));
  add(c, "mesh", "zb3_cell", L_CELL, (int64_t)ME * (K + 1));
  // state (2 time levels)
  add(c, "state", "u", L_EDGE, K, 2);
  add(c, "state", "w", L_CELL, K + 1, 2);
  add(c, "state", "theta_m", L_CELL, K, 2);
  add(c, "state", "rho_zz", L_CELL, K, 2);
  add(c, "state", "scalars", L_CELL, (int64_t)ns * K, 2);
  c.fields.back().nsub = ns;
  // diag
  for (const char* n : {"theta", "rho", "rho_base", "theta_base", "rho_p", "rho_p_save", "rho_pp",
                        "rho_zz_old_split", "rtheta_base", "rtheta_p", "rtheta_p_save", "rtheta_pp",
                        "rtheta_pp_old", "exner", "exner_base", "pressure_base", "pressure_p", "pressure", "h_divergence",
                        "kdiff", "ke", "divergence", "pv_cell", "tend_rtheta_adv", "cqw", "cofwr", "cofwz",
                        "cofwt", "a_tri", "alpha_tri", "gamma_tri"})
    add(c, "diag", n, L_CELL, K);
  add(c, "diag", "coftz", L_CELL, K + 1);
  add(c, "diag", "cofrz", L_NONE, K);
  for (const char* n : {"rw", "rw_p", "rw_save", "wwAvg", "wwAvg_split"}) add(c, "diag", n, L_CELL, K + 1);
  for (const char* n : {"ru", "ruAvg", "ruAvg_split", "ru_p", "ru_save", "cqu", "rho_edge", "v", "pv_edge",
                        "gradPVn", "gradPVt"})
    add(c, "diag", n, L_EDGE, K);
  for (const char* n : {"vorticity", "pv_vertex"}) add(c, "diag", n, L_VERTEX, K);
  for (const char* n : {"uReconstructX", "uReconstructY", "uReconstructZ", "uReconstructZonal",
                        "uReconstructMeridional"})
    add(c, "diag", n, L_CELL, K);
  // tend / tend_physics
  add(c, "tend", "u", L_EDGE, K);
  add(c, "tend", "u_euler", L_EDGE, K);
  add(c, "tend", "w", L_CELL, K + 1);
  add(c, "tend", "w_euler", L_CELL, K + 1);
  add(c, "tend", "theta_m", L_CELL, K);
  add(c, "tend", "theta_euler", L_CELL, K);
  add(c, "tend", "rho_zz", L_CELL, K);
  add(c, "tend", "rt_diabatic_tend", L_CELL, K);
  add(c, "tend", "scalars_tend", L_CELL, (int64_t)ns * K);
  c.fields.back().nsub = ns;
  add(c, "tend_physics", "rthdynten", L_CELL, K);
  // the lbc pool (mpas_atm_boundaries.F): time level 1 = tendency over the LBC interval, 2 = the
  // interval-end state; "dtr" = seconds from the step start to the interval end
  for (const char* n : {"lbc_u", "lbc_ru"}) add(c, "lbc", n, L_EDGE, K, 2);
  for (const char* n : {"lbc_rho_zz", "lbc_rtheta_m"}) add(c, "lbc", n, L_CELL, K, 2);
  add(c, "lbc", "lbc_scalars", L_CELL, (int64_t)ns * K, 2);
  c.fields.back().nsub = ns;
  add(c, "lbc", "dtr", L_NONE, 1);
  add(c, "scratch", "lbc_tmp", L_CELL, (int64_t)ns * K);
  // module scratch (mpas_atm_time_integration.F:35-71)
  // the physics tendencies of physics_get_tend (module scratch of the reference, 268-279), set by
  // the host when physics coupling is on (mpas_dyc_set_physics)
  add(c, "tend_physics", "rqvdynten", L_CELL, K);
  add(c, "tend_physics", "tend_rtheta_physics", L_CELL, K);
  add(c, "tend_physics", "tend_rho_physics", L_CELL, K);
  add(c, "tend_physics", "tend_ru_physics", L_EDGE, K);
  for (const char* n : {"qtot", "delsq_theta", "delsq_w",
                        "delsq_divergence", "dpdz", "s_max", "s_min", "rho_zz_int", "scalar_old_copy"})
    add(c, "scratch", n, L_CELL, K);
  for (const char* n : {"delsq_u", "ke_edge", "flux_arr", "flux_upwind_tmp", "flux_tmp",
                        "advflux_w", "advflux_th"})
    add(c, "scratch", n, L_EDGE, K);
  for (const char* n : {"delsq_vorticity", "ke_vertex"}) add(c, "scratch", n, L_VERTEX, K);
  add(c, "scratch", "horiz_flux_array", L_EDGE, (int64_t)ns * K);
  c.fields.back().nsub = ns;
  add(c, "scratch", "scale_arr", L_CELL, 2 * (int64_t)K);
  add(c, "scratch", "wdtn", L_CELL, K + 1);
  if (ns >= 2) {  // the second scalar of a pair in the monotone transport (advance_scalars_mono)
    for (const char* n : {"s_max_1", "s_min_1", "scalar_old_copy_1"}) add(c, "scratch", n, L_CELL, K);
    for (const char* n : {"flux_arr_1", "flux_upwind_tmp_1", "flux_tmp_1"}) add(c, "scratch", n, L_EDGE, K);
    add(c, "scratch", "scale_arr_1", L_CELL, 2 * (int64_t)K);
    add(c, "scratch", "wdtn_1", L_CELL, K + 1);
  }
  add(c, "scratch", "edge_bnd", L_EDGE, 1, 1, true);
  add(c, "scratch", "cell_bnd", L_CELL, 1, 1, true);
  add(c, "scratch", "bnd_edges", L_EDGE, 1, 1, true);
  add(c, "scratch", "bnd_pairs", L_EDGE, 1, 1, true);
  add(c, "scratch", "bnd_cells", L_CELL, 1, 1, true);
  add(c, "scratch", "cell_rec", L_CELL, CELL_REC, 1, true);
  add(c, "scratch", "cell_sdv", L_CELL, ME);
  add(c, "scratch", "zb_p", L_CELL, (int64_t)ME * (K + 1));
  add(c, "scratch", "zb_m", L_CELL, (int64_t)ME * (K + 1));
  // the saves srk3 rotates instead of copying (rotate_saves)
  for (const char* n : {"ru", "rw", "rtheta_p", "rho_p"}) {
    const int a = c.by_name[std::string("diag.") + n], b = c.by_name[std::string("diag.") + n + "_save"];
    c.fields[a].rot = b;
    c.fields[b].rot = a;
  }
  // inputs of the model-init precompute (mpas_dyc_model_init), allocated when set
  add(c, "mesh", "deriv_two", L_EDGE, 30);
  add(c, "mesh", "zb", L_EDGE, 2 * (int64_t)(K + 1));
  add(c, "mesh", "zb3", L_EDGE, 2 * (int64_t)(K + 1));
  add(c, "mesh", "meshDensity", L_CELL, 1);
  add(c, "mesh", "areaCell", L_CELL, 1);
  add(c, "mesh", "areaTriangle", L_VERTEX, 1);
  // optional: the C library's values of the two transcendental functions of the precompute, which the
  // caller computes as the compiled reference does (meshDensity**0.25 per cell and per edge midpoint,
  // the damping layer's sin per cell and level); unset, the device uses correctly rounded ones
  add(c, "mesh", "meshDensity_root4", L_CELL, 1);
  add(c, "mesh", "meshDensityEdge_root4", L_EDGE, 1);
  add(c, "mesh", "dss_sin", L_CELL, K);
  // inputs of the reconstruction coefficients (mpas_dyc_init_reconstruct), allocated when set
  for (const char* n : {"xCell", "yCell", "zCell"}) add(c, "mesh", n, L_CELL, 1);
  for (const char* n : {"xEdge", "yEdge", "zEdge"}) add(c, "mesh", n, L_EDGE, 1);
  for (const char* n : {"deriv_two", "zb", "zb3", "meshDensity", "areaCell", "areaTriangle", "xCell", "yCell", "zCell",
                        "xEdge", "yEdge", "zEdge", "meshDensity_root4", "meshDensityEdge_root4", "dss_sin"})
    c.fields[c.by_name[std::string("mesh.") + n]].lazy = true;
  // the maxEdges- and maxEdges2-strided mesh arrays (pack_mesh)
  for (const char* n : {"edgesOnCell", "cellsOnCell", "verticesOnCell", "kiteForCell", "coeffs_reconstruct",
                        "edgesOnCell_sign", "defc_a", "defc_b", "zb_cell", "zb3_cell"})
    c.fields[c.by_name[std::string("mesh.") + n]].me = 1;
  for (const char* n : {"edgesOnEdge", "weightsOnEdge"}) c.fields[c.by_name[std::string("mesh.") + n]].me = 2;
}

Field* find(Block& b, const char* pool, const char* name) {
  auto it = b.by_name.find(std::string(pool) + "." + name);
  if (it == b.by_name.end()) return nullptr;
  return &b.fields[it->second];
}

// state fields swap time levels every step; the lbc pool's two levels are fixed (tendency, state)
int slot_of(const mpas_dyc_ctx* c, const Field& f, int tl) {
  if (f.ntl == 2 && f.pool == "lbc") return tl == 2 ? 1 : 0;
  return (f.ntl == 2) ? ((tl == 2) ? 1 - c->cur : c->cur) : 0;
}

template <class T>
T* P(mpas_dyc_ctx* c, Block& b, const char* pool, const char* name, int tl = 1) {
  Field* f = find(b, pool, name);
  if (!f) {
    fprintf(stderr, "mpas_dycore: internal: missing field %s.%s\n", pool, name);
    abort();
  }
  return (T*)(f->packed ? f->packed : f->buf[slot_of(c, *f, tl)]);
}

Ptrs make_ptrs(mpas_dyc_ctx* c, Block& b) {
  Ptrs p{};
#define MI(x) p.x = P<const int>(c, b, "mesh", #x)
#define MR(x) p.x = P<const double>(c, b, "mesh", #x)
#define DG(x) p.x = P<double>(c, b, "diag", #x)
#define SC(x) p.x = P<double>(c, b, "scratch", #x)
  MI(nEdgesOnCell); MI(edgesOnCell); MI(cellsOnCell); MI(verticesOnCell); MI(kiteForCell);
  MI(cellsOnEdge); MI(verticesOnEdge); MI(nEdgesOnEdge); MI(edgesOnEdge); MI(nAdvCellsForEdge);
  MI(advCellsForEdge); MI(cellsOnVertex); MI(edgesOnVertex);
  MR(dcEdge); MR(dvEdge); MR(invDcEdge); MR(invDvEdge); MR(invAreaCell); MR(invAreaTriangle);
  MR(fEdge); MR(fVertex); MR(meshScalingDel2); MR(meshScalingDel4); MR(specZoneMaskEdge); MR(specZoneMaskCell);
  MR(fzm); MR(fzp); MR(rdzw); MR(rdzu);
  MR(edgesOnCell_sign); MR(edgesOnVertex_sign); MR(kiteAreasOnVertex); MR(weightsOnEdge);
  MR(adv_coefs); MR(adv_coefs_3rd); MR(defc_a); MR(defc_b);
  MR(zgrid); MR(zz); MR(zxu); MR(dss); MR(zb_cell); MR(zb3_cell);
  MR(u_init); MR(v_init); MR(t_init); MR(angleEdge);
  MR(latCell); MR(lonCell); MR(coeffs_reconstruct);
  DG(uReconstructX); DG(uReconstructY); DG(uReconstructZ); DG(uReconstructZonal); DG(uReconstructMeridional);
  p.u1 = P<double>(c, b, "state", "u", 1); p.u2 = P<double>(c, b, "state", "u", 2);
  p.w1 = P<double>(c, b, "state", "w", 1); p.w2 = P<double>(c, b, "state", "w", 2);
  p.theta_m1 = P<double>(c, b, "state", "theta_m", 1); p.theta_m2 = P<double>(c, b, "state", "theta_m", 2);
  p.rho_zz1 = P<double>(c, b, "state", "rho_zz", 1); p.rho_zz2 = P<double>(c, b, "state", "rho_zz", 2);
  p.scalars1 = P<double>(c, b, "state", "scalars", 1); p.scalars2 = P<double>(c, b, "state", "scalars", 2);
  DG(theta); DG(rho); DG(rho_base); DG(theta_base); DG(rho_p); DG(rho_p_save); DG(rho_pp); DG(rho_zz_old_split);
  DG(rtheta_base); DG(rtheta_p); DG(rtheta_p_save); DG(rtheta_pp); DG(rtheta_pp_old);
  DG(exner); DG(exner_base); DG(pressure_base); DG(pressure_p); DG(pressure); DG(h_divergence); DG(kdiff); DG(ke); DG(divergence);
  DG(pv_cell); DG(tend_rtheta_adv); DG(cqw); DG(cofwr); DG(cofwz); DG(cofwt); DG(coftz); DG(a_tri); DG(alpha_tri);
  DG(gamma_tri); DG(cofrz);
  DG(rw); DG(rw_p); DG(rw_save); DG(wwAvg); DG(wwAvg_split);
  DG(ru); DG(ruAvg); DG(ruAvg_split); DG(ru_p); DG(ru_save); DG(cqu); DG(rho_edge); DG(v); DG(pv_edge);
  DG(gradPVn); DG(gradPVt); DG(vorticity); DG(pv_vertex);
  p.tend_u = P<double>(c, b, "tend", "u"); p.tend_u_euler = P<double>(c, b, "tend", "u_euler");
  p.tend_w = P<double>(c, b, "tend", "w"); p.tend_w_euler = P<double>(c, b, "tend", "w_euler");
  p.tend_theta = P<double>(c, b, "tend", "theta_m"); p.tend_theta_euler = P<double>(c, b, "tend", "theta_euler");
  p.tend_rho = P<double>(c, b, "tend", "rho_zz"); p.rt_diabatic_tend = P<double>(c, b, "tend", "rt_diabatic_tend");
  p.scalars_tend = P<double>(c, b, "tend", "scalars_tend"); p.rthdynten = P<double>(c, b, "tend_physics", "rthdynten");
  SC(qtot);
  p.tend_ru_physics = P<double>(c, b, "tend_physics", "tend_ru_physics");
  p.tend_rtheta_physics = P<double>(c, b, "tend_physics", "tend_rtheta_physics");
  p.tend_rho_physics = P<double>(c, b, "tend_physics", "tend_rho_physics");
  p.rqvdynten = P<double>(c, b, "tend_physics", "rqvdynten");
  SC(delsq_theta); SC(delsq_w); SC(delsq_divergence); SC(delsq_u); SC(delsq_vorticity); SC(dpdz);
  SC(ke_vertex); SC(ke_edge); SC(horiz_flux_array);
  SC(s_max); SC(s_min); SC(scale_arr); SC(flux_arr); SC(flux_upwind_tmp); SC(flux_tmp); SC(wdtn); SC(rho_zz_int);
  SC(scalar_old_copy);
  SC(advflux_w); SC(advflux_th);
  p.edge_bnd = P<const int>(c, b, "scratch", "edge_bnd");
  p.cell_bnd = P<const int>(c, b, "scratch", "cell_bnd");
  p.bnd_edges = P<const int>(c, b, "scratch", "bnd_edges");
  p.bnd_pairs = P<const int>(c, b, "scratch", "bnd_pairs");
  p.bnd_cells = P<const int>(c, b, "scratch", "bnd_cells");
  p.cell_rec = P<const int>(c, b, "scratch", "cell_rec");
  p.cell_sdv = P<const double>(c, b, "scratch", "cell_sdv");
  p.zb_p = P<const double>(c, b, "scratch", "zb_p");
  p.zb_m = P<const double>(c, b, "scratch", "zb_m");
  MI(bdyMaskCell); MI(bdyMaskEdge); MI(nearestRelaxationCell);
  MR(meshScalingRegionalCell); MR(meshScalingRegionalEdge);
  p.lbc_u_t = P<const double>(c, b, "lbc", "lbc_u", 1); p.lbc_u_s = P<const double>(c, b, "lbc", "lbc_u", 2);
  p.lbc_ru_t = P<const double>(c, b, "lbc", "lbc_ru", 1); p.lbc_ru_s = P<const double>(c, b, "lbc", "lbc_ru", 2);
  p.lbc_rho_zz_t = P<const double>(c, b, "lbc", "lbc_rho_zz", 1);
  p.lbc_rho_zz_s = P<const double>(c, b, "lbc", "lbc_rho_zz", 2);
  p.lbc_rtheta_m_t = P<const double>(c, b, "lbc", "lbc_rtheta_m", 1);
  p.lbc_rtheta_m_s = P<const double>(c, b, "lbc", "lbc_rtheta_m", 2);
  p.lbc_scalars_t = P<const double>(c, b, "lbc", "lbc_scalars", 1);
  p.lbc_scalars_s = P<const double>(c, b, "lbc", "lbc_scalars", 2);
  p.lbc_dtr = P<const double>(c, b, "lbc", "dtr");
  SC(lbc_tmp);
  p.rw_rd = p.rw;
  p.w2_rd = p.w2;
  p.rho_zz2_rd = p.rho_zz2;
  // 0-d mesh fields are mirrored on the host
  p.cf1 = b.fields[b.by_name["mesh.cf1"]].buf[1] ? *(double*)b.fields[b.by_name["mesh.cf1"]].buf[1] : 0.0;
  p.cf2 = b.fields[b.by_name["mesh.cf2"]].buf[1] ? *(double*)b.fields[b.by_name["mesh.cf2"]].buf[1] : 0.0;
  p.cf3 = b.fields[b.by_name["mesh.cf3"]].buf[1] ? *(double*)b.fields[b.by_name["mesh.cf3"]].buf[1] : 0.0;
#undef MI
#undef MR
#undef DG
#undef SC
  return p;
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK)); }
#ifndef DIVDAMP_EPW
#define DIVDAMP_EPW 2  // edges per wavefront in k_divdamp
#endif

#define LAUNCH_E(kern, n, ...)                                                                             \
  do {                                                                                                     \
    if ((n) > 0 && !ctx->planning)                                                                         \
      hipLaunchKernelGGL(kern, dim3((unsigned)(((n) + EDGE_WPB - 1) / EDGE_WPB)), dim3(EDGE_THREADS), 0,    \
                         ctx->stream, __VA_ARGS__);                                                        \
  } while (0)
// a pair-layout kernel in its even-K or odd-K instance (its last template parameter, ODD)
// over n elements (PAIR_EPW per wavefront, PAIR_WPB wavefronts per workgroup)
#define LAUNCH_P(kern, n, ...)                                                                             \
  do {                                                                                                     \
    const int64_t nw_ = ((int64_t)(n) + PAIR_EPW - 1) / PAIR_EPW;                                           \
    if (nw_ > 0 && !ctx->planning)                                                                         \
      hipLaunchKernelGGL(kern, dim3((unsigned)((nw_ + PAIR_WPB - 1) / PAIR_WPB)), dim3(PAIR_THREADS), 0,    \
                         ctx->stream, __VA_ARGS__);                                                        \
  } while (0)
#define LAUNCH_PE(kern_even, kern_odd, n, ...)        \
  do {                                               \
    if (d.K & 1) LAUNCH_P(kern_odd, n, __VA_ARGS__);   \
    else LAUNCH_P(kern_even, n, __VA_ARGS__);          \
  } while (0)
#define LAUNCH(kern, n, ...)                                                                               \
  do {                                                                                                     \
    if ((n) > 0 && !ctx->planning)                                                                         \
      hipLaunchKernelGGL(kern, grid_for(n), dim3(BLOCK_THREADS), 0, ctx->stream, __VA_ARGS__);             \
  } while (0)

// ---------------------------------------------------------------------------
// halo exchange (mpas_dmpar_exch_halo_field, framework/mpas_dmpar.F)
// ---------------------------------------------------------------------------
bool needs_exchange(const mpas_dyc_ctx* ctx) { return ctx->blk.size() > 1 || ctx->nranks > 1 || ctx->loopback; }

// An exchange plan holds the fields' buffers, so its key names them: the time level and, per field,
// which of the buffers that the step's rotations move it is (buffer index of block 0)
std::string plan_key(mpas_dyc_ctx* ctx, const std::vector<XField>& fs) {
  std::string k = std::to_string(ctx->cur) + (ctx->plain_exchange ? "plain" : "");
  for (const auto& f : fs) {
    k += "|" + std::string(f.pool) + "." + f.name + "." + std::to_string(f.tl) + "." + std::to_string(f.layers);
    Field* F = ctx->blk.empty() ? nullptr : find(ctx->blk[0], f.pool, f.name);
    if (F && F->rot >= 0) k += "@" + std::to_string(F->rot_pos);
    else if (F && F->ntl == 2 && F->pool == "state") k += "@" + std::to_string(slot_of(ctx, *F, f.tl) ^ F->flip);
  }
  return k;
}

const XList* find_list(const Block& b, int loc, int layer, int dir, int peer_rank, int peer_block) {
  for (const auto& x : b.xl)
    if (x.loc == loc && x.layer == layer && x.dir == dir && x.peer_rank == peer_rank && x.peer_block == peer_block)
      return &x;
  return nullptr;
}

void free_plan(XPlan& pl) {
  for (void* p : pl.p2p_mapped) (void)hipIpcCloseMemHandle(p);
  for (void* p : {(void*)pl.d_pre, (void*)pl.d_post, (void*)pl.sendbuf, (void*)pl.recvbuf, (void*)pl.p2p_cnt,
                  (void*)pl.d_get, (void*)pl.d_ready, (void*)pl.d_cons})
    if (p) (void)hipFree(p);
  for (void* p : pl.pack_mem) (void)hipFree(p);
  for (void* p : pl.pull_mem) (void)hipFree(p);
  for (void* p : {(void*)pl.d_local, (void*)pl.d_pseg, (void*)pl.d_peer, (void*)pl.d_chunk})
    if (p) (void)hipFree(p);
  pl = XPlan{};
}

// captured steps bake pointers, list lengths and flags in: drop them when any of those changes
void drop_graphs(mpas_dyc_ctx* ctx) {
  for (auto& kv : ctx->graphs)
    if (kv.second) (void)hipGraphExecDestroy(kv.second);
  ctx->graphs.clear();
  ctx->graph_dt.clear();
}

void invalidate_plans(mpas_dyc_ctx* ctx) {
  if (!ctx->host_only) (void)hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->plans) free_plan(kv.second);
  ctx->plans.clear();
  ctx->planned.clear();
  drop_graphs(ctx);
}

bool is_local(const mpas_dyc_ctx* ctx, int peer_rank) { return peer_rank == ctx->rank && !ctx->rccl_local; }

std::vector<std::pair<int, int>> peers_of(const Block& b, int dir) {
  std::vector<std::pair<int, int>> peers;
  for (const auto& x : b.xl)
    if (x.dir == dir && x.n > 0 && x.peer_block >= 0) peers.emplace_back(x.peer_rank, x.peer_block);
  std::sort(peers.begin(), peers.end());
  peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
  return peers;
}

inline bool batched(const Dims& d);
inline bool pair_layout(const Dims& d);
bool split_phase(const mpas_dyc_ctx* ctx);

// Message layout: per block, peers in (rank, block) order; per peer, the fields in call
// order and per field the halo layers in ascending order (both sides agree on it).
int build_plan(mpas_dyc_ctx* ctx, const std::vector<XField>& fs, XPlan& pl) {
  const int nb = (int)ctx->blk.size();
  std::vector<XSeg> pre, post;
  std::vector<int64_t> pre_off, post_off;  // buffer offsets, patched once the buffers exist (-1: direct)
  std::vector<const std::vector<int32_t>*> pre_hidx;  // host send list of each block-pair pre segment
  int64_t stotal = 0, rtotal = 0;
  // the fused pack applies to the per-sub-step exchange (diag rtheta_pp [+ rho_pp], halo layer 1)
  bool fusable = !fs.empty() && fs.size() <= 2 && !ctx->plain_exchange;
  for (const auto& f : fs)
    fusable = fusable && std::string(f.pool) == "diag" && f.layers == 0x1u &&
              (std::string(f.name) == "rtheta_pp" || std::string(f.name) == "rho_pp");
  struct PackSeg { int block, is_rho; const XList* sx; size_t seg; };
  std::vector<PackSeg> pack_segs, unpack_segs;
  // the 876-887 exchange (rw_p, ru_p, rho_pp all layers, rtheta_pp layer 2) is fused into the stage's
  // last cell phase and damping (pack) and the halo recovery (unpack): XPack / XUnpack, dycore.h
  std::function<int(const XField&)> rec_fid = [](const XField& f) -> int {
    const std::string n(f.name);
    if (std::string(f.pool) != "diag") return -1;
    if (n == "rw_p" && f.layers == ALL_LAYERS) return 0;
    if (n == "rho_pp" && f.layers == ALL_LAYERS) return 1;
    if (n == "rtheta_pp" && f.layers == 0x2u) return 2;
    if (n == "ru_p" && f.layers == ALL_LAYERS) return 0;  // the edge field
    return -1;
  };
  // 1: the 876-887 exchange; 2: the tend_u exchange (642), packed by the stage's final tend_u kernel
  // (k_dyn_edges_p with finalize, k_dyn_edges_rk1b_b) and unpacked by k_smlstep_pert_b
  int fkind = 0;
  if (!ctx->plain_exchange && fs.size() == 4) {
    fkind = 1;
    for (const auto& f : fs) fkind = rec_fid(f) >= 0 ? fkind : 0;
  } else if (!ctx->plain_exchange && fs.size() == 1 && std::string(fs[0].pool) == "tend" &&
             std::string(fs[0].name) == "u" && fs[0].layers == 0x1u) {
    fkind = 2;
  } else if (!ctx->plain_exchange && !ctx->lbc && fs.size() == 1 && std::string(fs[0].pool) == "state" &&
             std::string(fs[0].name) == "u" && fs[0].tl == 2 && fs[0].layers == ALL_LAYERS) {
    fkind = 3;  // the u exchange after the recovery (988); regional runs overwrite u after the recovery
  }
  if (fkind >= 2) rec_fid = [](const XField&) -> int { return 0; };
  bool recfuse = fkind != 0;
  struct RecSeg { int block, fid; Loc loc; const XList* x; size_t seg; };
  std::vector<RecSeg> rec_pack, rec_unpack;
  auto field_of = [&](Block& b, const XField& f) -> Field* {
    Field* F = find(b, f.pool, f.name);
    if (!F || F->is_int || F->loc == L_NONE || (!F->buf[0] && !ctx->host_only)) {
      ctx->err = std::string("halo exchange of unsupported field ") + f.pool + "." + f.name;
      return nullptr;
    }
    return F;
  };
  for (int bi = 0; bi < nb; ++bi) {
    Block& b = ctx->blk[bi];
    for (const auto& pr : peers_of(b, MPAS_DYC_SEND)) {
      const bool local = is_local(ctx, pr.first);
      if (local && (pr.second < 0 || pr.second >= nb)) {
        ctx->err = "exchange list names block " + std::to_string(pr.second) + " not in this process";
        return MPAS_DYC_EINVAL;
      }
      const int64_t start = stotal;
      for (const auto& f : fs) {
        Field* F = field_of(b, f);
        if (!F) return MPAS_DYC_EINVAL;
        for (int layer = 1; layer <= 3; ++layer) {
          if (!((f.layers >> (layer - 1)) & 1u)) continue;
          const XList* sx = find_list(b, (int)F->loc, layer, MPAS_DYC_SEND, pr.first, pr.second);
          if (!sx || sx->n == 0) continue;
          const XList* rx = nullptr;
          Field* PF = nullptr;
          if (local) {
            Block& pb = ctx->blk[pr.second];
            rx = find_list(pb, (int)F->loc, layer, MPAS_DYC_RECV, ctx->rank, bi);
            if (!rx || rx->n != sx->n) {
              ctx->err = "send/recv lists of blocks " + std::to_string(bi) + "->" + std::to_string(pr.second) +
                         " disagree";
              return MPAS_DYC_EINVAL;
            }
            PF = find(pb, f.pool, f.name);
          }
          // a scalar-major field moves as nsub fields of inner/nsub doubles
          const int64_t sub_inner = F->inner / F->nsub;
          for (int is = 0; is < F->nsub; ++is) {
            XSeg sg{};
            sg.src = (const double*)F->buf[slot_of(ctx, *F, f.tl)] + (size_t)is * nloc(b, F->loc) * sub_inner;
            sg.sidx = sx->d_idx;
            sg.n = sx->n;
            sg.inner = (int)sub_inner;
            if (local) {
              sg.dst = (double*)PF->buf[slot_of(ctx, *PF, f.tl)] + (size_t)is * nloc(ctx->blk[pr.second], PF->loc) * sub_inner;
              sg.didx = rx->d_idx;
              pre_off.push_back(-1);
              fusable = false;  // a direct copy would reach the peer's halo before its cell phase reads it
              recfuse = false;
            } else {
              sg.didx = nullptr;
              pre_off.push_back(stotal);
              stotal += (int64_t)sx->n * sub_inner;
              if (fusable) pack_segs.push_back(PackSeg{bi, std::string(f.name) == "rho_pp" ? 1 : 0, sx, pre.size()});
              if (recfuse) rec_pack.push_back(RecSeg{bi, rec_fid(f), F->loc, sx, pre.size()});
            }
            pre.push_back(sg);
            pre_hidx.push_back(&sx->h_idx);
          }
          pl.maxn_pre = std::max(pl.maxn_pre, sx->n);
        }
      }
      if (!local && stotal > start) pl.rsend.push_back(XMsg{bi, pr.first, pr.second, start, stotal - start});
    }
    for (const auto& pr : peers_of(b, MPAS_DYC_RECV)) {
      const bool local = is_local(ctx, pr.first);
      const int64_t start = rtotal;
      for (const auto& f : fs) {
        Field* F = field_of(b, f);
        if (!F) return MPAS_DYC_EINVAL;
        for (int layer = 1; layer <= 3; ++layer) {
          if (!((f.layers >> (layer - 1)) & 1u)) continue;
          const XList* rx = find_list(b, (int)F->loc, layer, MPAS_DYC_RECV, pr.first, pr.second);
          if (!rx || rx->n == 0) continue;
          if (local) {  // filled by the sender's direct copy; check that one exists
            const XList* sx = (pr.second >= 0 && pr.second < nb)
                                  ? find_list(ctx->blk[pr.second], (int)F->loc, layer, MPAS_DYC_SEND, ctx->rank, bi)
                                  : nullptr;
            if (!sx || sx->n != rx->n) {
              ctx->err = "send/recv lists of blocks " + std::to_string(pr.second) + "->" + std::to_string(bi) +
                         " disagree";
              return MPAS_DYC_EINVAL;
            }
            continue;
          }
          const int64_t sub_inner = F->inner / F->nsub;
          for (int is = 0; is < F->nsub; ++is) {
            XSeg sg{};
            sg.sidx = nullptr;
            sg.dst = (double*)F->buf[slot_of(ctx, *F, f.tl)] + (size_t)is * nloc(b, F->loc) * sub_inner;
            sg.didx = rx->d_idx;
            sg.n = rx->n;
            sg.inner = (int)sub_inner;
            if (fusable) unpack_segs.push_back(PackSeg{bi, std::string(f.name) == "rho_pp" ? 1 : 0, rx, post.size()});
            if (recfuse) rec_unpack.push_back(RecSeg{bi, rec_fid(f), F->loc, rx, post.size()});
            post.push_back(sg);
            post_off.push_back(rtotal);
            rtotal += (int64_t)rx->n * sub_inner;
          }
          pl.maxn_post = std::max(pl.maxn_post, rx->n);
        }
      }
      if (!local && rtotal > start) pl.rrecv.push_back(XMsg{bi, pr.first, pr.second, start, rtotal - start});
    }
  }
  bool positional = false;
  // positional lists (mpas_dyc_set_exchange_positions): per peer rank one message, laid out as
  // mpas_dmpar lays out its buffer (mpas_dmpar.F:5448-5535): per field, per halo layer a region whose
  // slots the blocks of this process fill at their positions; the receiver reads its blocks' slots
  // at theirs.  Region sizes are the largest position over the blocks (both sides agree: it is one
  // buffer).  No fused pack / unpack for them.
  {
    std::set<int> pos_ranks;
    for (const auto& b : ctx->blk)
      for (const auto& x : b.xl)
        if (x.peer_block < 0 && x.n > 0) pos_ranks.insert(x.peer_rank);
    for (int dir = MPAS_DYC_SEND; dir <= MPAS_DYC_RECV; ++dir)
      for (int pr : pos_ranks) {
        int64_t& total = dir == MPAS_DYC_SEND ? stotal : rtotal;
        const int64_t start = total;
        for (const auto& f : fs) {
          Field* F0 = field_of(ctx->blk[0], f);
          if (!F0) return MPAS_DYC_EINVAL;
          for (int layer = 1; layer <= 3; ++layer) {
            if (!((f.layers >> (layer - 1)) & 1u)) continue;
            std::vector<const XList*> lx(nb, nullptr);
            int64_t npos = 0;
            for (int bi = 0; bi < nb; ++bi)
              for (const auto& x : ctx->blk[bi].xl)
                if (x.peer_block < 0 && x.n > 0 && x.peer_rank == pr && x.dir == dir && x.loc == (int)F0->loc &&
                    x.layer == layer) {
                  lx[bi] = &x;
                  for (int32_t q : x.h_pos) npos = std::max<int64_t>(npos, (int64_t)q + 1);
                }
            if (!npos) continue;
            const int64_t sub_inner = F0->inner / F0->nsub;
            for (int is = 0; is < F0->nsub; ++is) {
              for (int bi = 0; bi < nb; ++bi) {
                if (!lx[bi]) continue;
                Block& b = ctx->blk[bi];
                Field* F = field_of(b, f);
                if (!F) return MPAS_DYC_EINVAL;
                double* fld = (double*)F->buf[slot_of(ctx, *F, f.tl)] + (size_t)is * nloc(b, F->loc) * sub_inner;
                XSeg sg{};
                sg.n = lx[bi]->n;
                sg.inner = (int)sub_inner;
                if (dir == MPAS_DYC_SEND) {
                  sg.src = fld;
                  sg.sidx = lx[bi]->d_idx;
                  sg.didx = lx[bi]->d_pos;
                  pre.push_back(sg);
                  pre_off.push_back(total);
                  pl.maxn_pre = std::max(pl.maxn_pre, sg.n);
                } else {
                  sg.sidx = lx[bi]->d_pos;
                  sg.dst = fld;
                  sg.didx = lx[bi]->d_idx;
                  post.push_back(sg);
                  post_off.push_back(total);
                  pl.maxn_post = std::max(pl.maxn_post, sg.n);
                }
              }
              total += npos * sub_inner;
            }
          }
        }
        if (total > start) (dir == MPAS_DYC_SEND ? pl.rsend : pl.rrecv).push_back(XMsg{-1, pr, -1, start, total - start});
      }
    if (!pos_ranks.empty()) {
      positional = true;
      fusable = false;
      recfuse = false;
      for (const auto& m : pl.rsend)
        for (const auto& m2 : pl.rsend)
          if (m.peer_rank == m2.peer_rank && (m.block < 0) != (m2.block < 0)) {
            ctx->err = "rank " + std::to_string(m.peer_rank) + " has both positional and block-pair exchange lists";
            return MPAS_DYC_EINVAL;
          }
    }
  }
  if ((!pl.rsend.empty() || !pl.rrecv.empty()) && !ctx->comm && !(ctx->host_allgather && ctx->p2p) &&
      !ctx->host_only) {
    ctx->err = "exchange lists name other processes but no communicator was set (mpas_dyc_comm_init)";
    return MPAS_DYC_ECOMM;
  }
  // point-to-point messages between two ranks match in issue order: order both sides by
  // (source block, destination block)
  std::sort(pl.rsend.begin(), pl.rsend.end(), [](const XMsg& a, const XMsg& b) {
    return std::make_tuple(a.peer_rank, a.block, a.peer_block) < std::make_tuple(b.peer_rank, b.block, b.peer_block);
  });
  std::sort(pl.rrecv.begin(), pl.rrecv.end(), [](const XMsg& a, const XMsg& b) {
    return std::make_tuple(a.peer_rank, a.peer_block, a.block) < std::make_tuple(b.peer_rank, b.peer_block, b.block);
  });
  // One RCCL message per peer rank, as mpas_dmpar packs one buffer per processor for all its
  // blocks (mpas_dmpar.F:5386-5552): the block-pair messages to one rank are laid out back to back
  // in the order both sides sort them above, and go as one send / one receive.  (With one block
  // per rank nothing changes; with several, e.g. bench.py --blocks B or --rccl-local, the group
  // holds one message per peer rank instead of one per block pair.)
  auto merge_by_rank = [](std::vector<XMsg>& msgs, std::vector<int64_t>& offs) {
    std::map<int64_t, int64_t> base;  // message start, old layout -> new layout
    int64_t cur = 0;
    for (const XMsg& m : msgs) {
      base[m.off] = cur;
      cur += m.count;
    }
    for (int64_t& o : offs) {
      if (o < 0) continue;  // a direct in-process copy
      auto it = std::prev(base.upper_bound(o));
      o = it->second + (o - it->first);
    }
    std::vector<XMsg> merged;
    for (XMsg m : msgs) {
      m.off = base[m.off];
      if (!merged.empty() && merged.back().peer_rank == m.peer_rank) {
        merged.back().count += m.count;
        merged.back().block = merged.back().peer_block = -1;  // several block pairs
      } else {
        merged.push_back(m);
      }
    }
    msgs.swap(merged);
  };
  merge_by_rank(pl.rsend, pre_off);
  merge_by_rank(pl.rrecv, post_off);
  if (ctx->host_only) return MPAS_DYC_OK;  // the dry run keeps the message lists only
  if (ctx->loopback) stotal = rtotal = stotal + rtotal;  // rccl_group's loopback pairs stay inside
  // with other ranks, every exchange point is a one-sided one on every rank, messages or not: the
  // set-up numbers the exchange points in the same order on every rank (flag indices, records)
  pl.p2p = ctx->p2p && (!pl.rsend.empty() || !pl.rrecv.empty() || ctx->nranks > 1);
  pl.pull = pl.p2p && ctx->p2p_pull && !positional && !split_phase(ctx);
  if (pl.pull)
    if (const char* bk = getenv("MPAS_DYCORE_P2P_BUFFERS")) {  // debugging: these exchange points (key substrings) in buffers mode
      const std::string key = plan_key(ctx, fs), list = bk;
      size_t a = 0;
      while (a <= list.size()) {
        size_t e = list.find(',', a);
        if (e == std::string::npos) e = list.size();
        if (e > a && key.find(list.substr(a, e - a)) != std::string::npos) pl.pull = false;
        a = e + 1;
      }
    }
  if (pl.pull) {
    // the receiver copies from the fields: no buffers, and the kernels store and read the fields
    // themselves (no fused pack / unpack)
    fusable = recfuse = false;
    pl.h_pre = pre;
    pl.h_pre_off = pre_off;
    pl.h_pre_idx = pre_hidx;
    pl.h_post = post;
    pl.h_post_off = post_off;
    std::vector<XSeg> loc;
    for (size_t i = 0; i < pre.size(); ++i)
      if (pre_off[i] < 0) {
        loc.push_back(pre[i]);
        pl.maxn_local = std::max(pl.maxn_local, pre[i].n);
      }
    pl.nlocal = (int)loc.size();
    if (pl.nlocal) {
      HIPCHK(hipMalloc(&pl.d_local, loc.size() * sizeof(XSeg)));
      HIPCHK(hipMemcpy(pl.d_local, loc.data(), loc.size() * sizeof(XSeg), hipMemcpyHostToDevice));
    }
    return MPAS_DYC_OK;
  }
  if (pl.p2p) {
    // read by the peers (IPC): ordinary device memory, as the fields a pull reads -- the producer's
    // stores reach memory when its kernel ends (the L2 write-back that makes them visible to the
    // other XCDs), and the peers load it with system-scope loads (an uncached allocation here was
    // read stale by a peer process now and then: halo.hip)
    HIPCHK(hipMalloc(&pl.sendbuf, std::max<int64_t>(stotal, 1) * sizeof(double) + 256));
  } else if (stotal) {
    HIPCHK(hipMalloc(&pl.sendbuf, stotal * sizeof(double)));
  }
  // 256 B of slack: a fused unpack (ld_pp) reads the two levels of its lane's pair, one past the
  // last column at an odd K
  if (rtotal) HIPCHK(hipMalloc(&pl.recvbuf, rtotal * sizeof(double) + 256));
  for (size_t i = 0; i < pre.size(); ++i)
    if (pre_off[i] >= 0) pre[i].dst = pl.sendbuf + pre_off[i];
  for (size_t i = 0; i < post.size(); ++i) post[i].src = pl.recvbuf + post_off[i];
  pl.npre = (int)pre.size();
  pl.npost = (int)post.size();
  if (fusable && !pack_segs.empty()) {
    for (int bi = 0; bi < nb; ++bi) fusable = fusable && batched(ctx->blk[bi].d);
  }
  if (fusable && !pack_segs.empty()) {
    // per block: CSR over owned cells of (rtheta_pp slot, rho_pp slot) pairs; a cell has one
    // slot per RCCL peer that needs it (element i of a peer's list in both fields' segments)
    const bool with_rho = fs.size() == 2;
    pl.pack.assign(nb, PackMap{});
    for (int bi = 0; bi < nb; ++bi) {
      const Dims& d = ctx->blk[bi].d;
      std::map<std::pair<const XList*, int>, std::pair<double*, double*>> slot;  // (list, i) -> (rt, rho)
      for (const PackSeg& ps : pack_segs) {
        if (ps.block != bi) continue;
        for (int i = 0; i < ps.sx->n; ++i) {
          double* col = pre[ps.seg].dst + (size_t)i * pre[ps.seg].inner;
          auto& e = slot[{ps.sx, i}];
          (ps.is_rho ? e.second : e.first) = col;
        }
      }
      std::vector<std::vector<std::pair<double*, double*>>> per_cell(d.nCellsSolve);
      for (const auto& kv : slot) per_cell[kv.first.first->h_idx[kv.first.second]].push_back(kv.second);
      std::vector<int> start(d.nCellsSolve + 1, 0);
      std::vector<double*> rt, rho;
      for (int c = 0; c < d.nCellsSolve; ++c) {
        start[c] = (int)rt.size();
        for (const auto& e : per_cell[c]) {
          rt.push_back(e.first);
          rho.push_back(e.second);
        }
      }
      start[d.nCellsSolve] = (int)rt.size();
      if (rt.empty()) continue;
      int* d_start = nullptr;
      double** d_rt = nullptr;
      double** d_rho = nullptr;
      HIPCHK(hipMalloc(&d_start, start.size() * sizeof(int)));
      HIPCHK(hipMemcpy(d_start, start.data(), start.size() * sizeof(int), hipMemcpyHostToDevice));
      HIPCHK(hipMalloc(&d_rt, rt.size() * sizeof(double*)));
      HIPCHK(hipMemcpy(d_rt, rt.data(), rt.size() * sizeof(double*), hipMemcpyHostToDevice));
      pl.pack_mem.push_back(d_start);
      pl.pack_mem.push_back(d_rt);
      if (with_rho) {
        HIPCHK(hipMalloc(&d_rho, rho.size() * sizeof(double*)));
        HIPCHK(hipMemcpy(d_rho, rho.data(), rho.size() * sizeof(double*), hipMemcpyHostToDevice));
        pl.pack_mem.push_back(d_rho);
      }
      pl.pack[bi] = PackMap{d_start, d_rt, d_rho};
    }
    pl.fused_pack = ctx->fused_pack_enabled;
    // unpack maps: halo cell -> its columns in the receive buffer (consumers: pair kernels only)
    bool pair_all = true;
    for (int bi = 0; bi < nb; ++bi) pair_all = pair_all && pair_layout(ctx->blk[bi].d);
    if (pair_all && !unpack_segs.empty() && ctx->fused_pack_enabled) {
      pl.unpack.assign(nb, UnpackMap{});
      for (int bi = 0; bi < nb; ++bi) {
        const Dims& d = ctx->blk[bi].d;
        const int nh = d.nCells - d.nCellsSolve;
        std::vector<int> rt(nh, -1), rho(nh, -1);
        bool any = false;
        for (const PackSeg& ps : unpack_segs) {
          if (ps.block != bi) continue;
          for (int i = 0; i < ps.sx->n; ++i) {
            const int64_t off = (int64_t)(post[ps.seg].src - pl.recvbuf) + (int64_t)i * post[ps.seg].inner;
            (ps.is_rho ? rho : rt)[ps.sx->h_idx[i] - d.nCellsSolve] = (int)off;
            any = true;
          }
        }
        if (!any) continue;
        int *d_rt = nullptr, *d_rho = nullptr;
        HIPCHK(hipMalloc(&d_rt, std::max(nh, 1) * sizeof(int)));
        HIPCHK(hipMemcpy(d_rt, rt.data(), nh * sizeof(int), hipMemcpyHostToDevice));
        pl.pack_mem.push_back(d_rt);
        if (with_rho) {
          HIPCHK(hipMalloc(&d_rho, std::max(nh, 1) * sizeof(int)));
          HIPCHK(hipMemcpy(d_rho, rho.data(), nh * sizeof(int), hipMemcpyHostToDevice));
          pl.pack_mem.push_back(d_rho);
        }
        pl.unpack[bi] = UnpackMap{pl.recvbuf, d_rt, d_rho};
      }
      pl.fused_unpack = true;
    }
  }
  if (recfuse && (!rec_pack.empty() || !rec_unpack.empty()) && ctx->fused_pack_enabled) {
    bool pair_all = true;
    for (int bi = 0; bi < nb; ++bi) pair_all = pair_all && pair_layout(ctx->blk[bi].d);
    if (pair_all) {
      auto upload = [&](const void* h, size_t bytes, void** dptr) -> int {
        HIPCHK(hipMalloc(dptr, std::max<size_t>(bytes, 4)));
        if (bytes) HIPCHK(hipMemcpy(*dptr, h, bytes, hipMemcpyHostToDevice));
        pl.pack_mem.push_back(*dptr);
        return MPAS_DYC_OK;
      };
      pl.rpk_cell.assign(nb, XPack{});
      pl.rpk_edge.assign(nb, XPack{});
      pl.rup_cell.assign(nb, XUnpack{});
      pl.rup_edge.assign(nb, XUnpack{});
      for (int bi = 0; bi < nb; ++bi) {
        const Dims& d = ctx->blk[bi].d;
        for (const Loc loc : {L_CELL, L_EDGE}) {
          const int nsolve = loc == L_CELL ? d.nCellsSolve : d.nEdgesSolve;
          const int nh = (loc == L_CELL ? d.nCells : d.nEdges) - nsolve;
          const int nf = loc == L_CELL ? 3 : 1;
          // pack: per owned element, (field, send-buffer column) slots in element order
          std::vector<std::vector<std::pair<int, double*>>> per(nsolve);
          for (const RecSeg& rs : rec_pack) {
            if (rs.block != bi || rs.loc != loc) continue;
            for (int i = 0; i < rs.x->n; ++i)
              per[rs.x->h_idx[i]].emplace_back(rs.fid, pre[rs.seg].dst + (size_t)i * pre[rs.seg].inner);
          }
          std::vector<int> start(nsolve + 1, 0), fid;
          std::vector<double*> dst;
          for (int i = 0; i < nsolve; ++i) {
            start[i] = (int)fid.size();
            for (const auto& sl : per[i]) {
              fid.push_back(sl.first);
              dst.push_back(sl.second);
            }
          }
          start[nsolve] = (int)fid.size();
          if (!fid.empty()) {
            void *ds = nullptr, *df = nullptr, *dd = nullptr;
            CHK(upload(start.data(), start.size() * sizeof(int), &ds));
            CHK(upload(fid.data(), fid.size() * sizeof(int), &df));
            CHK(upload(dst.data(), dst.size() * sizeof(double*), &dd));
            (loc == L_CELL ? pl.rpk_cell : pl.rpk_edge)[bi] = XPack{(const int*)ds, (const int*)df, (double* const*)dd};
          }
          // unpack: per field and halo element, its column in the receive buffer
          std::vector<int> off((size_t)nf * std::max(nh, 0), -1);
          bool any = false;
          for (const RecSeg& rs : rec_unpack) {
            if (rs.block != bi || rs.loc != loc) continue;
            for (int i = 0; i < rs.x->n; ++i) {
              off[(size_t)rs.fid * nh + (rs.x->h_idx[i] - nsolve)] =
                  (int)((post[rs.seg].src - pl.recvbuf) + (int64_t)i * post[rs.seg].inner);
              any = true;
            }
          }
          const int* d_wb = nullptr;
          if (any && fkind == 3) {
            // each received halo edge is written back by one vertex of the block that has it among its
            // edgesOnVertex (the vertex kernel is its first reader); an edge without one: no fusion
            const Block& b = ctx->blk[bi];
            std::vector<int> wb(std::max(nh, 0), -1);
            bool ok = (int64_t)b.h_voe.size() >= 2LL * d.nEdges && (int64_t)b.h_eov.size() >= 3LL * d.nVertices;
            for (int i = 0; ok && i < nh; ++i) {
              if (off[i] < 0) continue;
              const int e = nsolve + i;
              for (int j = 0; j < 2 && wb[i] < 0; ++j) {
                const int v = b.h_voe[2 * (size_t)e + j];
                if (v < 0 || v >= d.nVertices) continue;
                for (int m = 0; m < 3; ++m)
                  if (b.h_eov[3 * (size_t)v + m] == e) wb[i] = v;
              }
              ok = wb[i] >= 0;
            }
            if (!ok) {
              recfuse = false;
              break;
            }
            void* dwb = nullptr;
            CHK(upload(wb.data(), wb.size() * sizeof(int), &dwb));
            d_wb = (const int*)dwb;
          }
          if (any) {
            void* doff = nullptr;
            CHK(upload(off.data(), off.size() * sizeof(int), &doff));
            (loc == L_CELL ? pl.rup_cell : pl.rup_edge)[bi] = XUnpack{pl.recvbuf, (const int*)doff, nh, d_wb};
          }
        }
      }
      if (recfuse) {
        pl.fused_rec = fkind;
        pl.fused_pack = pl.fused_unpack = true;
      } else {  // a write-back vertex is missing: the pack / unpack kernels run (maps unused)
        pl.rpk_cell.clear();
        pl.rpk_edge.clear();
        pl.rup_cell.clear();
        pl.rup_edge.clear();
      }
    }
  }
  if (pl.npre) {
    HIPCHK(hipMalloc(&pl.d_pre, pre.size() * sizeof(XSeg)));
    HIPCHK(hipMemcpy(pl.d_pre, pre.data(), pre.size() * sizeof(XSeg), hipMemcpyHostToDevice));
  }
  if (pl.npost) {
    HIPCHK(hipMalloc(&pl.d_post, post.size() * sizeof(XSeg)));
    HIPCHK(hipMemcpy(pl.d_post, post.data(), post.size() * sizeof(XSeg), hipMemcpyHostToDevice));
  }
  return MPAS_DYC_OK;
}

// a profile event pair's first half on `s` (the second is prof_mark_end); nothing unless profiling
int prof_mark(mpas_dyc_ctx* ctx, std::vector<hipEvent_t>& v, hipStream_t s) {
  if (!ctx->profile || ctx->planning) return MPAS_DYC_OK;
  hipEvent_t e = nullptr;
  HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventRecord(e, s));
  v.push_back(e);
  return MPAS_DYC_OK;
}

void set_last_key(mpas_dyc_ctx* ctx, const std::string& k) {
  const size_t n = std::min(k.size(), sizeof(ctx->last_key) - 1);
  memcpy(ctx->last_key, k.data(), n);
  ctx->last_key[n] = 0;
}

// The RCCL group of an exchange: one send and one receive per peer rank.  Loopback (timing
// emulation): each peer's pair goes to this rank itself; a send to self and the receive that
// matches it must have one size, so both move min(send, receive) doubles.
int rccl_group(mpas_dyc_ctx* ctx, const XPlan& pl) {
  NCCLCHK(ncclGroupStart());
  if (ctx->loopback) {
    // one self pair per peer rank of max(send, receive) doubles (a peer this rank only sends to or
    // only receives from gets one too); build_plan sizes both buffers for it
    std::map<int, std::pair<const XMsg*, const XMsg*>> peers;
    for (const XMsg& m : pl.rsend) peers[m.peer_rank].first = &m;
    for (const XMsg& m : pl.rrecv) peers[m.peer_rank].second = &m;
    for (const auto& kv : peers) {
      const XMsg *sm = kv.second.first, *rm = kv.second.second;
      const size_t n = (size_t)std::max(sm ? sm->count : 0, rm ? rm->count : 0);
      if (ctx->loopback == 2) {
        HIPCHK(hipMemcpyAsync(pl.recvbuf + (rm ? rm->off : 0), pl.sendbuf + (sm ? sm->off : 0), n * sizeof(double),
                              hipMemcpyDeviceToDevice, ctx->stream));
        continue;
      }
      NCCLCHK(ncclSend(pl.sendbuf + (sm ? sm->off : 0), n, ncclFloat64, ctx->rank, ctx->comm, ctx->stream));
      NCCLCHK(ncclRecv(pl.recvbuf + (rm ? rm->off : 0), n, ncclFloat64, ctx->rank, ctx->comm, ctx->stream));
    }
  } else {
    for (const XMsg& m : pl.rsend)
      NCCLCHK(ncclSend(pl.sendbuf + m.off, (size_t)m.count, ncclFloat64, m.peer_rank, ctx->comm, ctx->stream));
    for (const XMsg& m : pl.rrecv)
      NCCLCHK(ncclRecv(pl.recvbuf + m.off, (size_t)m.count, ncclFloat64, m.peer_rank, ctx->comm, ctx->stream));
  }
  NCCLCHK(ncclGroupEnd());
  return MPAS_DYC_OK;
}

// ---------------------------------------------------------------------------
// one-sided transfer set-up (MPAS_DYCORE_P2P, halo.hip): collective, outside graph capture
// ---------------------------------------------------------------------------
constexpr int P2P_MAX_POINTS = 4096;  // exchange points per context (a run builds ~60)

// nbytes from every rank, in rank order, over the library's communicator
int allgather_bytes(mpas_dyc_ctx* ctx, const void* mine, size_t nbytes, std::vector<char>& all) {
  all.assign(nbytes * ctx->nranks, 0);
  if (ctx->nranks == 1) {
    memcpy(all.data(), mine, nbytes);
    return MPAS_DYC_OK;
  }
  if (!ctx->comm && ctx->host_allgather) {
    if (ctx->host_allgather(mine, all.data(), (int64_t)nbytes, ctx->host_user) != 0) {
      ctx->err = "the host's all-gather (mpas_dyc_comm_init_host) failed";
      return MPAS_DYC_ECOMM;
    }
    return MPAS_DYC_OK;
  }
  char* d = nullptr;
  HIPCHK(hipMalloc(&d, nbytes * (ctx->nranks + 1)));
  const int r = [&]() -> int {
    HIPCHK(hipMemcpy(d, mine, nbytes, hipMemcpyHostToDevice));
    NCCLCHK(ncclAllGather(d, d + nbytes, nbytes, ncclUint8, ctx->comm, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(all.data(), d + nbytes, nbytes * ctx->nranks, hipMemcpyDeviceToHost));
    return MPAS_DYC_OK;
  }();
  (void)hipFree(d);
  return r;
}

// the node a rank runs on: IPC mappings exist only between processes of one node
uint64_t node_id() {
  char buf[512] = {0};
  (void)gethostname(buf, 255);
  if (FILE* f = fopen("/proc/sys/kernel/random/boot_id", "r")) {
    const size_t n = strlen(buf);
    if (!fgets(buf + n, (int)(sizeof(buf) - n - 1), f)) buf[n] = 0;
    fclose(f);
  }
  uint64_t h = 1469598103934665603ull;
  for (const char* c = buf; *c; ++c) h = (h ^ (unsigned char)*c) * 1099511628211ull;
  return h;
}

// p2p_init / p2p_setup return this when the one-sided transfer cannot run on some rank (IPC
// unsupported, ranks on several nodes, a mapping refused): every rank learns it from the same
// all-gathers, drops the transfer and plans again with RCCL (plan_all, p2p_fallback)
constexpr int P2P_UNAVAILABLE = 1;

// every rank's verdict on a local step of the set-up (collective): P2P_UNAVAILABLE on all ranks if
// any rank failed, with the first failing rank's reason in ctx->err
int p2p_vote(mpas_dyc_ctx* ctx, int local, const std::string& what) {
  int32_t mine = local == MPAS_DYC_OK ? 0 : 1;
  std::vector<char> all;
  CHK(allgather_bytes(ctx, &mine, sizeof(mine), all));
  for (int r = 0; r < ctx->nranks; ++r)
    if (((const int32_t*)all.data())[r]) {
      ctx->err = "one-sided transfer unavailable (" + what + " failed on rank " + std::to_string(r) +
                 (r == ctx->rank ? ": " + ctx->err : std::string()) + ")";
      return P2P_UNAVAILABLE;
    }
  return MPAS_DYC_OK;
}

// the flag arenas: this rank's, and every peer's mapped here
int p2p_init(mpas_dyc_ctx* ctx) {
  if (ctx->p2p_flags) return MPAS_DYC_OK;
  if (!ctx->comm && !ctx->host_allgather) {
    ctx->err = "MPAS_DYCORE_P2P: no communicator for the set-up (mpas_dyc_comm_init / _comm_init_host)";
    return MPAS_DYC_ECOMM;
  }
  int nr = ctx->nranks;
  if (ctx->loopback)  // the emulated peers are ranks the lists name, beyond this one-rank communicator
    for (const auto& b : ctx->blk)
      for (const auto& x : b.xl) nr = std::max(nr, x.peer_rank + 1);
  ctx->p2p_nr = nr;
  struct Rec {
    hipIpcMemHandle_t h;
    uint64_t node;
  } rec{};
  const int local = [&]() -> int {
    const size_t bytes = (size_t)P2P_MAX_POINTS * nr * 2 * sizeof(unsigned long long);
    HIPCHK(hipExtMallocWithFlags((void**)&ctx->p2p_flags, bytes, hipDeviceMallocUncached));
    HIPCHK(hipMemset(ctx->p2p_flags, 0, bytes));
    HIPCHK(hipMalloc(&ctx->p2p_status, sizeof(int)));
    HIPCHK(hipMemset(ctx->p2p_status, 0, sizeof(int)));
    HIPCHK(hipDeviceSynchronize());
    if (ctx->nranks > 1) HIPCHK(hipIpcGetMemHandle(&rec.h, ctx->p2p_flags));
    return MPAS_DYC_OK;
  }();
  ctx->p2p_peer_flags.assign(ctx->nranks, nullptr);
  ctx->p2p_peer_flags[ctx->rank] = ctx->p2p_flags;
  if (ctx->nranks == 1) return local;
  CHK(p2p_vote(ctx, local, "flag arena allocation"));
  rec.node = node_id();
  std::vector<char> all;
  CHK(allgather_bytes(ctx, &rec, sizeof(rec), all));
  for (int r = 0; r < ctx->nranks; ++r)
    if (((const Rec*)all.data())[r].node != rec.node) {
      ctx->err = "one-sided transfer unavailable (rank " + std::to_string(r) + " runs on another node)";
      return P2P_UNAVAILABLE;
    }
  const int opened = [&]() -> int {
    for (int r = 0; r < ctx->nranks; ++r) {
      if (r == ctx->rank) continue;
      void* p = nullptr;
      HIPCHK(hipIpcOpenMemHandle(&p, ((const Rec*)all.data())[r].h, hipIpcMemLazyEnablePeerAccess));
      ctx->p2p_mapped.push_back(p);
      ctx->p2p_peer_flags[r] = (unsigned long long*)p;
    }
    return MPAS_DYC_OK;
  }();
  return p2p_vote(ctx, opened, "mapping the peers' flag arenas");
}

// Maps the send buffers of the exchange points built since the last call and uploads their get /
// post tables.  Every rank builds the same exchange points in the same (plan key) order; the count
// is checked, and every message's size against its sender's.
int p2p_setup_pull(mpas_dyc_ctx* ctx, const std::vector<XPlan*>& todo);

int p2p_setup(mpas_dyc_ctx* ctx) {
  std::vector<XPlan*> todo, pulls;
  for (auto& kv : ctx->plans)
    if (kv.second.p2p && kv.second.p2p_id < 0) (kv.second.pull ? pulls : todo).push_back(&kv.second);
  // nothing to map and no peer process to agree with (a single block, or only in-process copies)
  if (todo.empty() && pulls.empty() && ctx->nranks == 1) return MPAS_DYC_OK;
  CHK(p2p_init(ctx));
  CHK(p2p_setup_pull(ctx, pulls));
  const int nr = ctx->nranks, me = ctx->rank;
  {
    int64_t n = (int64_t)todo.size();
    std::vector<char> all;
    CHK(allgather_bytes(ctx, &n, sizeof(n), all));
    for (int r = 0; r < nr; ++r)
      if (((const int64_t*)all.data())[r] != n) {
        ctx->err = "MPAS_DYCORE_P2P: rank " + std::to_string(r) + " built a different number of exchange points";
        return MPAS_DYC_ECOMM;
      }
  }
  if (todo.empty()) return MPAS_DYC_OK;
  // per exchange point: the send buffer's IPC handle, then per rank (offset, count) of the message to it
  const size_t per = sizeof(hipIpcMemHandle_t) + 2 * sizeof(int64_t) * nr;
  std::vector<char> mine(per * todo.size(), 0), all;
  const int handles = [&]() -> int {
    for (size_t i = 0; i < todo.size(); ++i) {
      char* r = mine.data() + per * i;
      if (nr > 1) HIPCHK(hipIpcGetMemHandle((hipIpcMemHandle_t*)r, todo[i]->sendbuf));
      int64_t* oc = (int64_t*)(r + sizeof(hipIpcMemHandle_t));
      for (int q = 0; q < nr; ++q) oc[2 * q] = oc[2 * q + 1] = -1;
      for (const XMsg& m : todo[i]->rsend) {
        if (m.peer_rank >= nr) continue;  // loopback: emulated ranks beyond the communicator
        oc[2 * m.peer_rank] = m.off;
        oc[2 * m.peer_rank + 1] = m.count;
      }
    }
    return MPAS_DYC_OK;
  }();
  if (nr > 1) CHK(p2p_vote(ctx, handles, "exporting the send buffers"));
  else CHK(handles);
  CHK(allgather_bytes(ctx, mine.data(), mine.size(), all));
  const int built = [&]() -> int {
    for (size_t i = 0; i < todo.size(); ++i) {
      XPlan& pl = *todo[i];
      if (ctx->p2p_next >= P2P_MAX_POINTS) {
        ctx->err = "MPAS_DYCORE_P2P: more than " + std::to_string(P2P_MAX_POINTS) + " exchange points";
        return MPAS_DYC_ESTATE;
      }
      pl.p2p_id = ctx->p2p_next++;
      auto flag = [&](unsigned long long* arena, int r, int k) {
        return arena + ((size_t)pl.p2p_id * ctx->p2p_nr + r) * 2 + k;
      };
      auto nchunk = [](int64_t n) { return (int)std::max<int64_t>(1, (n + P2P_CHUNK - 1) / P2P_CHUNK); };
      std::vector<P2PGet> gets;
      std::vector<unsigned long long*> ready;
      std::vector<const unsigned long long*> cons;
      if (ctx->loopback) {
        // as rccl_group: one pair per emulated peer of max(send, receive) doubles, all in this rank
        std::map<int, std::pair<const XMsg*, const XMsg*>> peers;
        for (const XMsg& m : pl.rsend) peers[m.peer_rank].first = &m;
        for (const XMsg& m : pl.rrecv) peers[m.peer_rank].second = &m;
        for (const auto& kv : peers) {
          const XMsg *sm = kv.second.first, *rm = kv.second.second;
          const int64_t n = std::max(sm ? sm->count : 0, rm ? rm->count : 0);
          gets.push_back(P2PGet{pl.sendbuf + (sm ? sm->off : 0), pl.recvbuf + (rm ? rm->off : 0), n,
                                flag(ctx->p2p_flags, kv.first, 0), flag(ctx->p2p_flags, kv.first, 1), nullptr,
                                nchunk(n)});
          ready.push_back(flag(ctx->p2p_flags, kv.first, 0));
          cons.push_back(flag(ctx->p2p_flags, kv.first, 1));
        }
      } else {
        for (const XMsg& m : pl.rsend) {
          ready.push_back(flag(ctx->p2p_peer_flags[m.peer_rank], me, 0));
          cons.push_back(flag(ctx->p2p_flags, m.peer_rank, 1));
        }
        for (const XMsg& m : pl.rrecv) {
          const char* rr = all.data() + (size_t)m.peer_rank * mine.size() + per * i;
          const int64_t* oc = (const int64_t*)(rr + sizeof(hipIpcMemHandle_t));
          if (oc[2 * me + 1] != m.count) {
            ctx->err = "MPAS_DYCORE_P2P: rank " + std::to_string(m.peer_rank) + " sends " +
                       std::to_string(oc[2 * me + 1]) + " doubles where this rank receives " + std::to_string(m.count);
            return MPAS_DYC_ECOMM;
          }
          const double* base = pl.sendbuf;
          if (m.peer_rank != me) {
            void* p = nullptr;
            HIPCHK(hipIpcOpenMemHandle(&p, *(const hipIpcMemHandle_t*)rr, hipIpcMemLazyEnablePeerAccess));
            pl.p2p_mapped.push_back(p);
            base = (const double*)p;
          }
          gets.push_back(P2PGet{base + oc[2 * me], pl.recvbuf + m.off, m.count, flag(ctx->p2p_flags, m.peer_rank, 0),
                                flag(ctx->p2p_peer_flags[m.peer_rank], me, 1), nullptr, nchunk(m.count)});
        }
      }
      if (cons.size() > 256 || ready.size() > 256) {
        ctx->err = "MPAS_DYCORE_P2P: more than 256 peers";
        return MPAS_DYC_EINVAL;
      }
      // [0] uses, [1 + i] chunks pulled from get peer i, [1 + nget] finished workgroups of k_p2p_exchange
      HIPCHK(hipMalloc(&pl.p2p_cnt, (2 + gets.size()) * sizeof(unsigned long long)));
      HIPCHK(hipMemset(pl.p2p_cnt, 0, (2 + gets.size()) * sizeof(unsigned long long)));
      for (size_t j = 0; j < gets.size(); ++j) {
        gets[j].done = pl.p2p_cnt + 1 + j;
        pl.get_chunks = std::max(pl.get_chunks, gets[j].nchunk);
      }
      pl.nget = (int)gets.size();
      pl.nready = (int)ready.size();
      pl.ncons = (int)cons.size();
      auto upload = [&](const void* h, size_t bytes, void** d) -> int {
        HIPCHK(hipMalloc(d, std::max<size_t>(bytes, 8)));
        if (bytes) HIPCHK(hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice));
        return MPAS_DYC_OK;
      };
      CHK(upload(gets.data(), gets.size() * sizeof(P2PGet), (void**)&pl.d_get));
      CHK(upload(ready.data(), ready.size() * sizeof(void*), (void**)&pl.d_ready));
      CHK(upload(cons.data(), cons.size() * sizeof(void*), (void**)&pl.d_cons));
    }
    return MPAS_DYC_OK;
  }();
  return nr > 1 ? p2p_vote(ctx, built, "mapping the peers' send buffers") : built;
}

// variable-size all-gather: every rank's bytes, in rank order
int allgatherv_bytes(mpas_dyc_ctx* ctx, const std::vector<char>& mine, std::vector<std::vector<char>>& out) {
  int64_t n = (int64_t)mine.size();
  std::vector<char> sizes;
  CHK(allgather_bytes(ctx, &n, sizeof(n), sizes));
  int64_t mx = 0;
  for (int r = 0; r < ctx->nranks; ++r) mx = std::max(mx, ((const int64_t*)sizes.data())[r]);
  std::vector<char> pad(mine);
  pad.resize(std::max<int64_t>(mx, 1), 0);
  std::vector<char> all;
  CHK(allgather_bytes(ctx, pad.data(), pad.size(), all));
  out.assign(ctx->nranks, {});
  for (int r = 0; r < ctx->nranks; ++r) {
    const char* b = all.data() + (size_t)r * pad.size();
    out[r].assign(b, b + ((const int64_t*)sizes.data())[r]);
  }
  return MPAS_DYC_OK;
}

// Pull plans: every rank exports, per exchange point and message, its pack segments (the field
// buffer -- IPC handle, mapped once per peer and buffer -- the sub-field offset, the send list);
// the receiver pairs them in message order with its unpack segments into k_p2p_pull's segments.
int p2p_setup_pull(mpas_dyc_ctx* ctx, const std::vector<XPlan*>& todo) {
  const int nr = ctx->nranks, me = ctx->rank;
  if (todo.empty()) return MPAS_DYC_OK;
  // the field buffer a pack segment reads
  auto base_of = [&](const double* p, size_t& bytes) -> const double* {
    for (const auto& b : ctx->blk)
      for (const auto& f : b.fields)
        for (int t = 0; t < f.ntl; ++t) {
          const char* q = (const char*)f.buf[t];
          if (!q || f.is_int) continue;
          const size_t nb = (size_t)field_bytes(b, f) + 256;
          if ((const char*)p >= q && (const char*)p < q + nb) {
            bytes = nb;
            return (const double*)q;
          }
        }
    return nullptr;
  };
  std::vector<char> rec;
  auto put = [&](const void* v, size_t n) { rec.insert(rec.end(), (const char*)v, (const char*)v + n); };
  std::vector<const double*> bases;
  std::map<const double*, int32_t> base_id;
  std::vector<char> body;
  const int exported = [&]() -> int {
    std::vector<char> hdr;
    for (XPlan* pp : todo) {
      const XPlan& pl = *pp;
      const int32_t nmsg = (int32_t)pl.rsend.size();
      body.insert(body.end(), (const char*)&nmsg, (const char*)&nmsg + 4);
      for (const XMsg& m : pl.rsend) {
        std::vector<size_t> segs;  // in buffer order: the receiver pairs them with its unpack segments so
        for (size_t i = 0; i < pl.h_pre.size(); ++i)
          if (pl.h_pre_off[i] >= m.off && pl.h_pre_off[i] < m.off + m.count) segs.push_back(i);
        std::sort(segs.begin(), segs.end(), [&](size_t a, size_t b) { return pl.h_pre_off[a] < pl.h_pre_off[b]; });
        const int32_t dest = m.peer_rank, ns = (int32_t)segs.size();
        body.insert(body.end(), (const char*)&dest, (const char*)&dest + 4);
        body.insert(body.end(), (const char*)&ns, (const char*)&ns + 4);
        for (size_t i : segs) {
          const XSeg& sg = pl.h_pre[i];
          size_t nb = 0;
          const double* b = base_of(sg.src, nb);
          if (!b) {
            ctx->err = "internal: pack segment outside every field";
            return MPAS_DYC_ESTATE;
          }
          if (!base_id.count(b)) {
            base_id[b] = (int32_t)bases.size();
            bases.push_back(b);
          }
          const int32_t id = base_id[b], n = sg.n, inner = sg.inner;
          const int64_t off = (const char*)sg.src - (const char*)b;
          const std::vector<int32_t>& idx = *pl.h_pre_idx[i];
          body.insert(body.end(), (const char*)&id, (const char*)&id + 4);
          body.insert(body.end(), (const char*)&off, (const char*)&off + 8);
          body.insert(body.end(), (const char*)&n, (const char*)&n + 4);
          body.insert(body.end(), (const char*)&inner, (const char*)&inner + 4);
          body.insert(body.end(), (const char*)idx.data(), (const char*)(idx.data() + n));
        }
      }
    }
    const int32_t nbase = (int32_t)bases.size();
    put(&nbase, 4);
    for (const double* b : bases) {
      const uint64_t a = (uint64_t)(uintptr_t)b;
      hipIpcMemHandle_t h{};
      if (nr > 1) HIPCHK(hipIpcGetMemHandle(&h, (void*)b));
      put(&a, 8);
      put(&h, sizeof(h));
    }
    rec.insert(rec.end(), body.begin(), body.end());
    return MPAS_DYC_OK;
  }();
  if (nr > 1) CHK(p2p_vote(ctx, exported, "exporting the field buffers"));
  else CHK(exported);
  std::vector<std::vector<char>> all;
  CHK(allgatherv_bytes(ctx, rec, all));
  // per rank: its buffer table and a cursor over its per-plan messages
  struct Reader {
    const char* p;
    std::vector<std::pair<uint64_t, hipIpcMemHandle_t>> bases;
  };
  std::vector<Reader> rd(nr);
  for (int r = 0; r < nr; ++r) {
    const char* p = all[r].data();
    int32_t nb;
    memcpy(&nb, p, 4);
    p += 4;
    for (int i = 0; i < nb; ++i) {
      std::pair<uint64_t, hipIpcMemHandle_t> e;
      memcpy(&e.first, p, 8);
      memcpy(&e.second, p + 8, sizeof(hipIpcMemHandle_t));
      p += 8 + sizeof(hipIpcMemHandle_t);
      rd[r].bases.push_back(e);
    }
    rd[r].p = p;
  }
  struct SegIn {
    int32_t id, n, inner;
    int64_t off;
    const int32_t* idx;
  };
  // a mapped field buffer of rank r (each buffer opened once per context)
  auto mapped = [&](int r, int32_t id, const double*& out) -> int {
    const auto& e = rd[r].bases.at(id);
    if (r == me) {
      out = (const double*)(uintptr_t)e.first;
      return MPAS_DYC_OK;
    }
    auto key = std::make_pair(r, e.first);
    auto it = ctx->p2p_fields.find(key);
    if (it == ctx->p2p_fields.end()) {
      void* p = nullptr;
      HIPCHK(hipIpcOpenMemHandle(&p, e.second, hipIpcMemLazyEnablePeerAccess));
      ctx->p2p_mapped.push_back(p);
      it = ctx->p2p_fields.emplace(key, p).first;
    }
    out = (const double*)it->second;
    return MPAS_DYC_OK;
  };
  const int built = [&]() -> int {
    for (XPlan* pp : todo) {
      XPlan& pl = *pp;
      if (ctx->p2p_next >= P2P_MAX_POINTS) {
        ctx->err = "MPAS_DYCORE_P2P: more than " + std::to_string(P2P_MAX_POINTS) + " exchange points";
        return MPAS_DYC_ESTATE;
      }
      pl.p2p_id = ctx->p2p_next++;
      auto flag = [&](unsigned long long* arena, int r, int k) {
        return arena + ((size_t)pl.p2p_id * ctx->p2p_nr + r) * 2 + k;
      };
      // every rank's messages of this exchange point: rank -> destination -> its pack segments
      std::vector<std::map<int, std::vector<SegIn>>> from(nr);
      for (int r = 0; r < nr; ++r) {
        const char*& q = rd[r].p;
        int32_t nmsg;
        memcpy(&nmsg, q, 4);
        q += 4;
        for (int m = 0; m < nmsg; ++m) {
          int32_t dest, ns;
          memcpy(&dest, q, 4);
          memcpy(&ns, q + 4, 4);
          q += 8;
          auto& v = from[r][dest];
          for (int k = 0; k < ns; ++k) {
            SegIn si{};
            memcpy(&si.id, q, 4);
            memcpy(&si.off, q + 4, 8);
            memcpy(&si.n, q + 12, 4);
            memcpy(&si.inner, q + 16, 4);
            si.idx = (const int32_t*)(q + 20);
            q += 20 + 4 * (size_t)si.n;
            v.push_back(si);
          }
        }
      }
      std::vector<P2PSeg> segs;
      std::vector<P2PPeer> peers;
      std::vector<unsigned long long*> ready;
      std::vector<const unsigned long long*> cons;
      std::map<int, int> peer_ix;
      auto peer_of = [&](int src) -> int {
        auto it = peer_ix.find(src);
        if (it != peer_ix.end()) return it->second;
        const int ix = (int)peers.size();
        peer_ix[src] = ix;
        const bool here = ctx->loopback || src == me;
        peers.push_back(P2PPeer{flag(ctx->p2p_flags, src, 0),
                                here ? flag(ctx->p2p_flags, src, 1) : flag(ctx->p2p_peer_flags[src], me, 1), nullptr, 0});
        return ix;
      };
      auto upload = [&](const void* h, size_t bytes) -> void* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
        if (bytes && hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) {
          (void)hipFree(d);
          return nullptr;
        }
        pl.pull_mem.push_back(d);
        return d;
      };
      std::set<int> loop_peers;  // loopback: every emulated peer
      for (const XMsg& m : pl.rrecv) {
        std::vector<size_t> mine_post;  // in buffer order, as the sender exported its pack segments
        for (size_t i = 0; i < pl.h_post.size(); ++i)
          if (pl.h_post_off[i] >= m.off && pl.h_post_off[i] < m.off + m.count) mine_post.push_back(i);
        std::sort(mine_post.begin(), mine_post.end(),
                  [&](size_t a, size_t b) { return pl.h_post_off[a] < pl.h_post_off[b]; });
        const int src = m.peer_rank;
        const int ix = peer_of(src);
        if (ctx->loopback) {
          // timing only: the peer's segments are this rank's own pack segments to that peer
          loop_peers.insert(src);
          std::vector<size_t> theirs;
          for (const XMsg& sm : pl.rsend)
            if (sm.peer_rank == src)
              for (size_t i = 0; i < pl.h_pre.size(); ++i)
                if (pl.h_pre_off[i] >= sm.off && pl.h_pre_off[i] < sm.off + sm.count) theirs.push_back(i);
          std::sort(theirs.begin(), theirs.end(), [&](size_t a, size_t b) { return pl.h_pre_off[a] < pl.h_pre_off[b]; });
          for (size_t k = 0; k < std::min(theirs.size(), mine_post.size()); ++k) {
            const XSeg &a = pl.h_pre[theirs[k]], &b = pl.h_post[mine_post[k]];
            const int n = std::min(a.n, b.n);
            segs.push_back(P2PSeg{a.src, b.dst, a.sidx, b.didx, n, std::min(a.inner, b.inner), ix});
          }
          continue;
        }
        auto f = from[src].find(me);
        if (f == from[src].end() || f->second.size() != mine_post.size()) {
          ctx->err = "MPAS_DYCORE_P2P: rank " + std::to_string(src) + "'s message to rank " + std::to_string(me) +
                     " does not match this rank's receive lists";
          return MPAS_DYC_ECOMM;
        }
        for (size_t k = 0; k < mine_post.size(); ++k) {
          const SegIn& a = f->second[k];
          const XSeg& b = pl.h_post[mine_post[k]];
          if (a.n != b.n || a.inner != b.inner) {
            ctx->err = "MPAS_DYCORE_P2P: rank " + std::to_string(src) + " sends " + std::to_string(a.n) +
                       " elements where rank " + std::to_string(me) + " receives " + std::to_string(b.n);
            return MPAS_DYC_ECOMM;
          }
          const double* base = nullptr;
          CHK(mapped(src, a.id, base));
          const int* sidx = (const int*)upload(a.idx, sizeof(int32_t) * (size_t)a.n);
          if (!sidx) {
            ctx->err = "hipMalloc for a peer's send list failed";
            return MPAS_DYC_EHIP;
          }
          segs.push_back(P2PSeg{(const double*)((const char*)base + a.off), b.dst, sidx, b.didx, a.n, a.inner, ix});
        }
      }
      if (ctx->loopback) {
        for (const XMsg& m : pl.rsend) {
          loop_peers.insert(m.peer_rank);
          (void)peer_of(m.peer_rank);
        }
        for (int q : loop_peers) ready.push_back(flag(ctx->p2p_flags, q, 0));
      } else {
        for (const XMsg& m : pl.rsend) {
          ready.push_back(flag(ctx->p2p_peer_flags[m.peer_rank], me, 0));
          cons.push_back(flag(ctx->p2p_flags, m.peer_rank, 1));
        }
      }
      std::vector<int2> chunks;
      for (size_t k = 0; k < segs.size(); ++k)
        for (int c = 0; c < segs[k].n; c += P2P_PULL_COLS) {
          chunks.push_back(make_int2((int)k, c));
          peers[segs[k].peer].nwg += 1;
        }
      pl.nchunk = (int)chunks.size();
      pl.npeer_work = 0;
      for (const P2PPeer& pr : peers) pl.npeer_work += pr.nwg ? 1 : 0;
      if (ctx->loopback)  // the emulated readers of this rank: the peers with segments here
        for (const P2PPeer& pr : peers)
          if (pr.nwg) cons.push_back(pr.consumed);
      if (cons.size() > 256 || ready.size() > 256) {
        ctx->err = "MPAS_DYCORE_P2P: more than 256 peers";
        return MPAS_DYC_EINVAL;
      }
      // [0] uses, [1] finished workgroups of k_p2p_pull, [2 + i] workgroups done for peer i
      HIPCHK(hipMalloc(&pl.p2p_cnt, (2 + peers.size()) * sizeof(unsigned long long)));
      HIPCHK(hipMemset(pl.p2p_cnt, 0, (2 + peers.size()) * sizeof(unsigned long long)));
      for (size_t j = 0; j < peers.size(); ++j) peers[j].done = pl.p2p_cnt + 2 + j;
      pl.npseg = (int)segs.size();
      pl.nready = (int)ready.size();
      pl.ncons = (int)cons.size();
      pl.d_pseg = (P2PSeg*)upload(segs.data(), segs.size() * sizeof(P2PSeg));
      pl.d_chunk = (int2*)upload(chunks.data(), chunks.size() * sizeof(int2));
      pl.d_peer = (P2PPeer*)upload(peers.data(), peers.size() * sizeof(P2PPeer));
      pl.d_ready = (unsigned long long**)upload(ready.data(), ready.size() * sizeof(void*));
      pl.d_cons = (const unsigned long long**)upload(cons.data(), cons.size() * sizeof(void*));
      if (!pl.d_pseg || !pl.d_chunk || !pl.d_peer || !pl.d_ready || !pl.d_cons) {
        ctx->err = "hipMalloc for a pull plan failed";
        return MPAS_DYC_EHIP;
      }
      // d_ready / d_cons are freed with the plan (free_plan); keep them out of pull_mem
      pl.pull_mem.erase(std::remove_if(pl.pull_mem.begin(), pl.pull_mem.end(),
                                       [&](void* q) { return q == (void*)pl.d_ready || q == (void*)pl.d_cons ||
                                                             q == (void*)pl.d_pseg || q == (void*)pl.d_peer ||
                                                             q == (void*)pl.d_chunk; }),
                        pl.pull_mem.end());
    }
    return MPAS_DYC_OK;
  }();
  return nr > 1 ? p2p_vote(ctx, built, "mapping the peers' fields") : built;
}

// the one-sided transfer dropped on every rank (P2P_UNAVAILABLE): its mappings and arena freed, the
// plans rebuilt for RCCL by the caller
void p2p_fallback(mpas_dyc_ctx* ctx) {
  fprintf(stderr, "mpas_dycore rank %d: %s; halo exchanges go through RCCL\n", ctx->rank, ctx->err.c_str());
  invalidate_plans(ctx);
  for (void* p : ctx->p2p_mapped) (void)hipIpcCloseMemHandle(p);
  ctx->p2p_mapped.clear();
  ctx->p2p_fields.clear();
  if (ctx->p2p_flags) (void)hipFree(ctx->p2p_flags);
  ctx->p2p_flags = nullptr;
  ctx->p2p_peer_flags.clear();
  ctx->p2p = 0;
}

// p2p_status: a wait of k_p2p_get that timed out
int p2p_check(mpas_dyc_ctx* ctx) {
  if (!ctx->p2p_status) return MPAS_DYC_OK;
  int st = 0;
  HIPCHK(hipMemcpy(&st, ctx->p2p_status, sizeof(int), hipMemcpyDeviceToHost));
  if (st) {
    ctx->err = std::string("MPAS_DYCORE_P2P: a peer's halo message did not arrive within 30 s (last exchange: ") +
               ctx->last_key + ")";
    return MPAS_DYC_ECOMM;
  }
  return MPAS_DYC_OK;
}

// part: 0 the whole exchange; with one-sided transfer a split-phase exchange runs as 1 (pack and
// post, at exchange_async) and 2 (get and unpack, at exchange_wait), all on the compute stream
int exchange(mpas_dyc_ctx* ctx, const std::vector<XField>& fs, int part = 0) {
  if (!needs_exchange(ctx)) return MPAS_DYC_OK;
  const std::string key = plan_key(ctx, fs);
  if (ctx->record) ctx->record->push_back(key);
  auto it = ctx->plans.find(key);
  if (it == ctx->plans.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (!ctx->host_only) (void)hipStreamIsCapturing(ctx->stream, &cs);
    if (cs != hipStreamCaptureStatusNone) {
      ctx->err = "internal: exchange plan missing during graph capture";
      return MPAS_DYC_ESTATE;
    }
    XPlan pl;
    int r = build_plan(ctx, fs, pl);
    if (r) {
      free_plan(pl);
      return r;
    }
    it = ctx->plans.emplace(key, std::move(pl)).first;
  }
  if (ctx->planning) return MPAS_DYC_OK;
  XPlan& pl = it->second;
  if (pl.p2p) {
    if (pl.p2p_id < 0) {  // built outside plan_all (mpas_dyc_halo_exchange): every rank is here too
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(ctx->stream, &cs);
      if (cs != hipStreamCaptureStatusNone) {
        ctx->err = "internal: one-sided exchange set up during graph capture";
        return MPAS_DYC_ESTATE;
      }
      const int r = p2p_setup(ctx);
      if (r == P2P_UNAVAILABLE) {  // every rank is here: this exchange, and the rest, through RCCL
        if (!ctx->comm) return MPAS_DYC_ECOMM;
        p2p_fallback(ctx);
        return exchange(ctx, fs, part);
      }
      CHK(r);
    }
    if (pl.pull) {  // blocking only (build_plan): the whole exchange at the first call
      if (part == 2) return MPAS_DYC_OK;
      CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
      if (pl.nlocal)
        hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_local + 3) / 4, pl.nlocal), dim3(256), 0, ctx->stream, pl.d_local);
      set_last_key(ctx, key);
      CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
      hipLaunchKernelGGL(k_p2p_pull, dim3(pl.nchunk + 1), dim3(256), 0, ctx->stream, (const P2PSeg*)pl.d_pseg,
                         (const int2*)pl.d_chunk, pl.nchunk, (const P2PPeer*)pl.d_peer, pl.npeer_work,
                         (unsigned long long* const*)pl.d_ready, pl.nready, (const unsigned long long* const*)pl.d_cons,
                         pl.ncons, pl.p2p_cnt, ctx->p2p_status);
      CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
      CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
      return MPAS_DYC_OK;
    }
    if (part == 0 && !ctx->p2p_merge) {  // the two launches (A/B of the merged one)
      CHK(exchange(ctx, fs, 1));
      return exchange(ctx, fs, 2);
    }
    if (part == 0) {  // blocking: post and get as one launch (k_p2p_exchange)
      CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
      if (pl.npre && !pl.fused_pack)
        hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_pre + 3) / 4, pl.npre), dim3(256), 0, ctx->stream, pl.d_pre);
      set_last_key(ctx, key);
      CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
      hipLaunchKernelGGL(k_p2p_exchange, dim3(std::max(pl.get_chunks, 1), pl.nget + 1), dim3(256), 0, ctx->stream,
                         (const P2PGet*)pl.d_get, pl.nget, (unsigned long long* const*)pl.d_ready, pl.nready,
                         (const unsigned long long* const*)pl.d_cons, pl.ncons, pl.p2p_cnt, ctx->p2p_status);
      CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
      if (pl.npost && !pl.fused_unpack)
        hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_post + 3) / 4, pl.npost), dim3(256), 0, ctx->stream, pl.d_post);
      CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
      return MPAS_DYC_OK;
    }
    if (part == 1) {
      if (pl.npre && !pl.fused_pack)
        hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_pre + 3) / 4, pl.npre), dim3(256), 0, ctx->stream, pl.d_pre);
      set_last_key(ctx, key);
      hipLaunchKernelGGL(k_p2p_post, dim3(1), dim3(64), 0, ctx->stream, pl.p2p_cnt, pl.d_ready, pl.nready);
    }
    if (part != 1) {
      CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
      hipLaunchKernelGGL(k_p2p_get, dim3(std::max(pl.get_chunks, 1), pl.nget + 1), dim3(256), 0, ctx->stream,
                         (const P2PGet*)pl.d_get, pl.nget, (const unsigned long long* const*)pl.d_cons, pl.ncons,
                         (const unsigned long long*)pl.p2p_cnt, ctx->p2p_status);
      CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
      if (pl.npost && !pl.fused_unpack)
        hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_post + 3) / 4, pl.npost), dim3(256), 0, ctx->stream, pl.d_post);
    }
    return MPAS_DYC_OK;
  }
  if (part == 2) return MPAS_DYC_OK;  // in-process copies only: done at part 1
  const bool whole = !ctx->in_async;  // a blocking exchange: all of it is exposed
  if (whole) CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
  if (pl.npre && !pl.fused_pack)
    hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_pre + 3) / 4, pl.npre), dim3(256), 0, ctx->stream, pl.d_pre);
  if (!pl.rsend.empty() || !pl.rrecv.empty()) {
    set_last_key(ctx, key);
    CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
    CHK(rccl_group(ctx, pl));
    CHK(prof_mark(ctx, ctx->prof_rccl, ctx->stream));
  }
  if (pl.npost && !pl.fused_unpack)
    hipLaunchKernelGGL(k_halo_copy, dim3((pl.maxn_post + 3) / 4, pl.npost), dim3(256), 0, ctx->stream, pl.d_post);
  if (whole) CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
  return MPAS_DYC_OK;
}

// The plan of an exchange whose pack the producing kernel does (XPlan::fused_pack), or nullptr
const XPlan* fused_pack_plan(mpas_dyc_ctx* ctx, const std::vector<XField>& fs) {
  if (ctx->planning || !needs_exchange(ctx)) return nullptr;
  auto it = ctx->plans.find(plan_key(ctx, fs));
  if (it == ctx->plans.end() || !it->second.fused_pack || it->second.pack.size() != ctx->blk.size()) return nullptr;
  return &it->second;
}

// The plan of the 876-887 or 642 exchange when its pack and unpack are fused (XPlan::fused_rec), or
// nullptr
const XPlan* fused_rec_plan(mpas_dyc_ctx* ctx, const std::vector<XField>& fs) {
  if (ctx->planning || !needs_exchange(ctx)) return nullptr;
  auto it = ctx->plans.find(plan_key(ctx, fs));
  if (it == ctx->plans.end() || !it->second.fused_rec || it->second.rpk_cell.size() != ctx->blk.size()) return nullptr;
  return &it->second;
}

// Kernel families: 0 "general" (one column per wave, loads where used -- any mesh), 1 "batched"
// (k_*_b / k_*_r: per-cell records, every load issued up front; maxEdges 6 or 7), 2 "pair"
// (k_*_p: two edges per wave, two levels per lane; even K).  All three give the same bits
// (tests/test_gpu_kernels.py); the environment variable MPAS_DYCORE_KERNELS=general|batched|pair,
// read when a context is created, caps the family (default pair).
int g_kernel_tier = 2;
// k_dyn_delsq_vc in the pair layout (MPAS_DYCORE_DELSQ_PAIR=0, read when a context is created: the
// batched kernel)
int g_delsq_pair = 1;
// k_dyn_cells2 in the pair layout (MPAS_DYCORE_CELLS2_PAIR=0: the batched kernel)
int g_cells2_pair = 1;
// k_dyn_cells1 in the pair layout (MPAS_DYCORE_CELLS1_PAIR=0: the batched kernel)
int g_cells1_pair = 1;
inline bool batched(const Dims& d) {
  return g_kernel_tier >= 1 && (d.maxEdges == 6 || d.maxEdges == 7) && d.maxEdges2 >= 2 * d.maxEdges - 2;
}


// atm_set_smlstep_pert_variables fused into the batched k_dyn_cells3_r for the cells without a halo
// edge (MPAS_DYCORE_FUSE_SMLSTEP=0, read when a context is created: the separate kernel for all)
int g_fuse_smlstep = 1;
inline bool fuse_smlstep(const Dims& d) { return g_fuse_smlstep && batched(d); }

// pair-layout edge kernels (k_*_p: two edges per wave, two levels per lane); at an odd K the last
// pair's second level is past the column: loaded (the 256 B of slack behind every field covers the
// last column), never stored, and every level-dependent expression masks it as it masks the
// levels above K at an even K
// (the wide build: one column per wavefront, K <= 2 x 64 - 1 levels, same kernels)
inline bool pair_layout(const Dims& d) { return g_kernel_tier >= 2 && batched(d) && d.K <= 64 * (3 - PAIR_EPW) - 1; }

// why a block cannot run regional LBCs (they need the pair layout), named by its actual cause
std::string lbc_layout_error(const Dims& d) {
  if (g_kernel_tier < 2) return "regional LBCs need the pair kernel family (MPAS_DYCORE_KERNELS=pair)";
  return "regional LBCs need cells of at most 7 edges (max(nEdgesOnCell) = " + std::to_string(d.maxEdges) +
         ") and maxEdges2 >= " + std::to_string(2 * d.maxEdges - 2);
}

// The kernels index the maxEdges-strided mesh arrays with the mesh's actual cell degree, not with
// the declared one.  maxEdges in a mesh file is "the largest number of neighbors that a primal mesh
// cell *may* have" (core_atmosphere/Registry.xml:13-16) -- MPAS-distributed meshes declare 10 (and
// maxEdges2 = 20) -- and the reference never reads a slot past nEdgesOnCell (its loops run to
// nEdgesOnCell, and edgesOnCell_sign is 0 there, mpas_atm_core.F:1025-1050).  So the block keeps the
// Fortran images at the declared strides (buf: set/get_field, the device pointers) and the kernels
// read copies at
//   maxEdges  = max(nEdgesOnCell) over the block, at least 6 (or the declared value, if smaller),
//   maxEdges2 = max(max(nEdgesOnEdge), 2 * maxEdges - 2), at most the declared value
// (2 maxEdges - 2 = the edgesOnEdge slots the batched kernels load, NE2).  The floor of 6 gives every
// block of an SCVT mesh (pentagons..heptagons) the same kernel family whatever its cells, so the
// blocks of different ranks make the same choices.  Every slot a kernel reads is a prefix of the
// declared row, so the packed copy holds the same values at the same (element, slot).
int pack_mesh(mpas_dyc_ctx* ctx, Block& b) {
  Dims& d = b.d;
  int me = std::min(6, b.me_decl), me2 = 0;
  for (int c = 0; c < d.nCells; ++c) me = std::max(me, b.h_noc[c]);
  if (me > b.me_decl) {
    ctx->err = "nEdgesOnCell exceeds maxEdges (" + std::to_string(me) + " > " + std::to_string(b.me_decl) + ")";
    return MPAS_DYC_EINVAL;
  }
  if ((int64_t)b.h_noe.size() >= d.nEdges) {
    for (int e = 0; e < d.nEdges; ++e) me2 = std::max(me2, b.h_noe[e]);
    if (me2 > b.me2_decl) {
      ctx->err = "nEdgesOnEdge exceeds maxEdges2 (" + std::to_string(me2) + " > " + std::to_string(b.me2_decl) + ")";
      return MPAS_DYC_EINVAL;
    }
    me2 = std::min(b.me2_decl, std::max(me2, 2 * me - 2));
  } else {
    me2 = b.me2_decl;  // nEdgesOnEdge not set: keep the declared stride
  }
  for (auto& f : b.fields) {
    if (!f.me) continue;
    const int64_t slot = f.inner / (f.me == 1 ? b.me_decl : b.me2_decl);
    const int64_t inner = slot * (f.me == 1 ? me : me2);
    const int64_t es = f.is_int ? 4 : 8, n = nloc(b, f.loc);
    if (inner == f.inner) {
      if (f.packed) (void)hipFree(f.packed);
      f.packed = nullptr;
      f.packed_inner = 0;
      continue;
    }
    if (f.packed && f.packed_inner != inner) {
      (void)hipFree(f.packed);
      f.packed = nullptr;
    }
    if (!f.packed) {
      HIPCHK(hipMalloc(&f.packed, n * inner * es + 256));
      HIPCHK(hipMemsetAsync(f.packed, 0, n * inner * es + 256, ctx->stream));
    }
    f.packed_inner = inner;
    HIPCHK(hipMemcpy2DAsync(f.packed, inner * es, f.buf[0], f.inner * es, inner * es, n, hipMemcpyDeviceToDevice,
                            ctx->stream));
  }
  if (d.maxEdges != me || d.maxEdges2 != me2) {
    d.maxEdges = me;
    d.maxEdges2 = me2;
    invalidate_plans(ctx);  // kernel families and the fused exchanges follow the strides
  }
  return MPAS_DYC_OK;
}

// Halo-boundary flags of the split-phase exchanges: an edge is "boundary" when one of its
// cells is a halo cell (it reads exchanged cell data); an owned cell is "boundary" when
// one of its edges is a halo edge (it reads exchanged edge data).
int compute_bnd(mpas_dyc_ctx* ctx) {
  for (auto& b : ctx->blk) {
    const Dims& d = b.d;
    if ((int64_t)b.h_coe.size() < 2LL * d.nEdges || (int64_t)b.h_eoc.size() < (int64_t)b.me_decl * d.nCells ||
        (int64_t)b.h_noc.size() < d.nCells) {
      ctx->err = "mesh connectivity (cellsOnEdge, edgesOnCell, nEdgesOnCell) not set";
      return MPAS_DYC_ESTATE;
    }
    CHK(pack_mesh(ctx, b));
    if (ctx->lbc && !pair_layout(d)) {
      ctx->err = lbc_layout_error(d);
      return MPAS_DYC_EINVAL;
    }
    std::vector<int32_t> eb(d.nEdges + 1, 1), cb(d.nCells + 1, 1);
    for (int e = 0; e < d.nEdges; ++e)
      eb[e] = (b.h_coe[2 * e] >= d.nCellsSolve || b.h_coe[2 * e + 1] >= d.nCellsSolve) ? 1 : 0;
    for (int c = 0; c < d.nCells; ++c) {
      int bnd = c >= d.nCellsSolve ? CELL_HALO_EDGE | CELL_BND_EDGE : 0;
      for (int i = 0; i < b.h_noc[c]; ++i) {
        const int e = b.h_eoc[(size_t)c * b.me_decl + i];
        if (e >= d.nEdgesSolve) bnd |= CELL_HALO_EDGE;
        if (e >= d.nEdges || eb[e]) bnd |= CELL_BND_EDGE;
      }
      cb[c] = bnd;
    }
    HIPCHK(hipMemcpy(find(b, "scratch", "edge_bnd")->buf[0], eb.data(), eb.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(find(b, "scratch", "cell_bnd")->buf[0], cb.data(), cb.size() * 4, hipMemcpyHostToDevice));
    std::vector<int32_t> le, lp, lc;
    for (int e = 0; e < d.nEdges; ++e) {
      if (!eb[e]) continue;
      le.push_back(e);
      if (b.h_coe[2 * e] < d.nCellsSolve || b.h_coe[2 * e + 1] < d.nCellsSolve) lp.push_back(e);
    }
    for (int c = 0; c < d.nCellsSolve; ++c)
      if (cb[c] & CELL_HALO_EDGE) lc.push_back(c);
    if (!le.empty())
      HIPCHK(hipMemcpy(find(b, "scratch", "bnd_edges")->buf[0], le.data(), le.size() * 4, hipMemcpyHostToDevice));
    if (!lp.empty())
      HIPCHK(hipMemcpy(find(b, "scratch", "bnd_pairs")->buf[0], lp.data(), lp.size() * 4, hipMemcpyHostToDevice));
    if (!lc.empty())
      HIPCHK(hipMemcpy(find(b, "scratch", "bnd_cells")->buf[0], lc.data(), lc.size() * 4, hipMemcpyHostToDevice));
    if (b.d.n_bnd_edges != (int)le.size() || b.d.n_bnd_pairs != (int)lp.size() || b.d.n_bnd_cells != (int)lc.size())
      drop_graphs(ctx);  // captured steps bake the list lengths into their launches
    b.d.n_bnd_edges = (int)le.size();
    b.d.n_bnd_pairs = (int)lp.size();
    b.d.n_bnd_cells = (int)lc.size();
    hipLaunchKernelGGL(k_build_cell_rec, dim3((d.nCells + 1 + 255) / 256), dim3(256), 0, ctx->stream, d,
                       P<const int>(ctx, b, "mesh", "nEdgesOnCell"), P<const int>(ctx, b, "mesh", "edgesOnCell"),
                       P<const int>(ctx, b, "mesh", "cellsOnEdge"), P<const double>(ctx, b, "mesh", "dvEdge"),
                       P<const double>(ctx, b, "mesh", "edgesOnCell_sign"), P<int>(ctx, b, "scratch", "cell_rec"),
                       P<double>(ctx, b, "scratch", "cell_sdv"));
    HIPCHK(hipGetLastError());
    {
      const int64_t n = (int64_t)(d.nCells + 1) * d.maxEdges * (d.K + 1);
      hipLaunchKernelGGL(k_build_zb, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 65536)), dim3(256), 0,
                         ctx->stream, n, P<const double>(ctx, b, "mesh", "zb_cell"),
                         P<const double>(ctx, b, "mesh", "zb3_cell"), P<double>(ctx, b, "scratch", "zb_p"),
                         P<double>(ctx, b, "scratch", "zb_m"));
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  ctx->bnd_ready = true;
  return MPAS_DYC_OK;
}

// Auto mode splits only when halo traffic goes through RCCL: block-to-block copies inside
// one GPU are a single short kernel, and splitting them only adds launches.
bool split_phase(const mpas_dyc_ctx* ctx) {
  if (!needs_exchange(ctx)) return false;
  if (ctx->overlap >= 0) return ctx->overlap != 0;
  if (ctx->p2p) return false;  // the transfer is the receiver's kernel: nothing to overlap it with
  return ctx->nranks > 1 || ctx->rccl_local || ctx->loopback;
}

// First half of a split-phase exchange: after everything queued on the compute stream,
// the exchange stream packs, talks RCCL and unpacks; exchange_wait joins it back.
int issue_async(mpas_dyc_ctx* ctx, const std::vector<XField>& fs) {
  HIPCHK(hipStreamWaitEvent(ctx->xstream, ctx->xfork, 0));
  hipStream_t s = ctx->stream;
  ctx->stream = ctx->xstream;  // exchange() issues on ctx->stream
  ctx->in_async = true;
  const int r = exchange(ctx, fs);
  ctx->in_async = false;
  ctx->stream = s;
  if (r) return r;
  HIPCHK(hipEventRecord(ctx->xjoin, ctx->xstream));
  return MPAS_DYC_OK;
}

int exchange_async(mpas_dyc_ctx* ctx, const std::vector<XField>& fs) {
  if (ctx->planning) return exchange(ctx, fs);
  if (ctx->p2p) {  // no second stream: pack and post now, the get at exchange_wait
    ctx->p2p_open = fs;
    ctx->p2p_pending = true;
    return exchange(ctx, fs, 1);
  }
  HIPCHK(hipEventRecord(ctx->xfork, ctx->stream));
  if (ctx->late_issue) {
    ctx->late_fs = fs;
    ctx->late_pending = true;
    return MPAS_DYC_OK;
  }
  return issue_async(ctx, fs);
}

int exchange_wait(mpas_dyc_ctx* ctx) {
  if (ctx->planning) return MPAS_DYC_OK;
  if (ctx->p2p_pending) {
    ctx->p2p_pending = false;
    CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
    CHK(exchange(ctx, ctx->p2p_open, 2));
    CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));
    return MPAS_DYC_OK;
  }
  if (ctx->late_pending) {
    ctx->late_pending = false;
    CHK(issue_async(ctx, ctx->late_fs));
  }
  CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));  // the compute stream's work before the join
  HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->xjoin, 0));
  CHK(prof_mark(ctx, ctx->prof_exposed, ctx->stream));  // ... completes once the join has
  return MPAS_DYC_OK;
}

// ---------------------------------------------------------------------------
// reference routines, one host function each (per block)
// ---------------------------------------------------------------------------
// The saves of atm_rk_integration_setup (1847-1850) and of atm_rk_dynamics_substep_finish
// (6051-6054) -- ru_save = ru, rw_save = rw, rtheta_p_save = rtheta_p, rho_p_save = rho_p -- are
// buffer rotations: X_save takes X's buffer, which holds exactly those values, and X takes the
// other one.  The first stage's recovery (2998-3059) overwrites X on every element before any
// kernel reads X again; until then the readers of X read X_save (stage_pre), which holds the same
// values bit for bit.
void rotate_saves(mpas_dyc_ctx* ctx) {
  for (auto& b : ctx->blk)
    for (const char* n : {"ru", "rw", "rtheta_p", "rho_p"}) {
      Field* x = find(b, "diag", n);
      Field* xs = &b.fields[x->rot];
      std::swap(x->buf[0], xs->buf[0]);
      x->rot_pos ^= 1;
      xs->rot_pos ^= 1;
    }
}

// theta_m_1 = theta_m_2 at the end of a dynamics substep (6058): the two time levels trade buffers;
// time level 2 then holds stale values until the next first-stage recovery, and its readers before
// that read time level 1 (stage_pre)
void swap_theta(mpas_dyc_ctx* ctx) {
  for (auto& b : ctx->blk) {
    Field* f = find(b, "state", "theta_m");
    std::swap(f->buf[0], f->buf[1]);
    f->flip ^= 1;
  }
}

// The pointers the kernels of a dynamics substep's first stage see until its recovery: X -> X_save
// for the rotated saves, time level 2 -> time level 1 of theta_m (swapped buffers) and, in the
// first dynamics substep, of u, w and rho_zz, whose copies of atm_rk_integration_setup (1852-1855)
// are not made either: the first stage's recovery writes time level 2 of all of them on every
// element (u: 3048-3059, w: 3013 and 3063-3097, rho_zz: 2998-3001 with the garbage slot, 2989-2991).
Ptrs stage_pre(const Ptrs& p0, bool first_substep) {
  Ptrs p = p0;
  p.ru = p.ru_save;
  p.rw = p.rw_save;
  p.rw_rd = p.rw_save;
  p.rtheta_p = p.rtheta_p_save;
  p.theta_m2 = p.theta_m1;
  if (first_substep) {
    p.u2 = p.u1;
    p.w2 = p.w1;
    p.w2_rd = p.w1;
    p.rho_zz2 = p.rho_zz1;
    p.rho_zz2_rd = p.rho_zz1;
  }
  return p;
}

// The first stage's last cell phase reads as stage_pre (rw_rd, w2_rd, rho_zz2_rd) but its fused
// recovery (k_acoustic_cells_r<ME, true>) writes the fields themselves
Ptrs stage_fin(const Ptrs& p0, bool first_substep) {
  Ptrs p = p0;
  p.rw_rd = p.rw_save;
  if (first_substep) {
    p.w2_rd = p.w1;
    p.rho_zz2_rd = p.rho_zz1;
  }
  return p;
}

// the rotations one atm_srk3 makes (rk_integration_setup + each substep_finish that is not the last)
int step_rotations(const Config& cf) { return cf.split_dynamics_transport ? cf.dynamics_split_steps : 1; }

// replay of a captured step: its rotations happened on the host at capture time; repeat them
void apply_step_rotations(mpas_dyc_ctx* ctx) {
  const int n = step_rotations(ctx->cf);
  if (n & 1) rotate_saves(ctx);
  if ((n - 1) & 1) swap_theta(ctx);
}

// the buffer layout a step starts from: time level parity and the rotations' positions
std::string layout_sig(mpas_dyc_ctx* ctx) {
  Block& b = ctx->blk[0];
  return std::to_string(ctx->cur) + "." + std::to_string(find(b, "diag", "ru")->rot_pos) + "." +
         std::to_string(find(b, "state", "theta_m")->flip);
}

// the rotated fields' buffers and positions, to undo the rotations of a dry run (plan_all)
struct Layout {
  std::vector<std::tuple<Field*, void*, void*, int, int>> f;
};
Layout save_layout(mpas_dyc_ctx* ctx) {
  Layout l;
  for (auto& b : ctx->blk)
    for (auto& f : b.fields)
      if (f.rot >= 0 || (f.pool == "state" && f.name == "theta_m")) l.f.emplace_back(&f, f.buf[0], f.buf[1], f.rot_pos, f.flip);
  return l;
}
void restore_layout(const Layout& l) {
  for (const auto& t : l.f) {
    Field* f = std::get<0>(t);
    f->buf[0] = std::get<1>(t);
    f->buf[1] = std::get<2>(t);
    f->rot_pos = std::get<3>(t);
    f->flip = std::get<4>(t);
  }
}

// atm_rk_integration_setup (1847-1857): the saves and the time level 2 copies are rotate_saves /
// stage_pre; scalars_2 = scalars_1 (1856) is copied over owned+halo elements (the scalar
// transport writes owned columns of time level 2 and exchanges the rest, and with scalar advection
// off time level 2 must hold the old values)
void rk_integration_setup(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p) {
  CopyList c{};
  c.src[0] = p.scalars1;
  c.dst[0] = p.scalars2;
  c.n[0] = (int64_t)(d.nCells + 1) * d.K * d.ns;
  const unsigned gx = (unsigned)std::min<int64_t>((c.n[0] + 255) / 256, 2048);
  if (!ctx->planning) hipLaunchKernelGGL(k_copy_many, dim3(gx, 1), dim3(256), 0, ctx->stream, c);
}


void vert_imp_coefs(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, double dts) {
  if (pair_layout(d))
    LAUNCH_PE((k_vert_imp_coefs_p<false>), (k_vert_imp_coefs_p<true>), std::max(d.nCellsSolve, 1), d, p, dts, ctx->cf.epssm);
  else
    LAUNCH(k_vert_imp_coefs, std::max(d.nCellsSolve, 1), d, p, dts, ctx->cf.epssm);
}

// part: 0 = all kernels; 1 = only k_dyn_cells1, which reads nothing the exchange after the
// diagnostics (1234-1249) or at the substep boundary (1282-1297) delivers; 2 = the rest
// hdiv_done: the previous stage's w recovery computed h_divergence (recover_cells3 with hdiv), so
// at rk_step 2 / 3, where k_dyn_cells1 computes nothing else, it is not launched
// tp: the block's pack map of the tend_u exchange that follows (642, XPlan::fused_rec), or none
void dyn_tend(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, int rk_step, double dt, int part = 0,
              bool hdiv_done = false, bool last = true, XPack tp = XPack{}) {
  const Config& cf = ctx->cf;
  DynTendScal s{};
  s.rk_step = rk_step;
  s.store_phys_diag = last ? 1 : 0;  // last: the dt's final dyn_tend
  s.dt = dt;
  s.invDt = 1.0 / dt;
  s.coef_3rd_order = cf.coef_3rd_order;
  s.c_s = cf.smagorinsky_coef;
  if (cf.horiz_mixing_smag) {
    s.h_mom_eddy_visc4 = cf.visc4_2dsmag * (cf.len_disp * cf.len_disp * cf.len_disp);
    s.h_theta_eddy_visc4 = s.h_mom_eddy_visc4;
  } else {
    s.h_mom_eddy_visc4 = cf.h_mom_eddy_visc4;
    s.h_theta_eddy_visc4 = cf.h_theta_eddy_visc4;
  }
  if (cf.rayleigh_damp_u)
    s.rayleigh_coef_inverse = 1.0 / ((double)cf.number_rayleigh_damp_u_levels *
                                     (cf.rayleigh_damp_u_timescale_days * SECONDS_PER_DAY));
  const bool bt = batched(d), m6 = d.maxEdges == 6;
  if (part != 2 && !(hdiv_done && rk_step > 1)) {
    if (!bt) LAUNCH(k_dyn_cells1, d.nCells, d, p, cf, s);
    else if (pair_layout(d) && g_cells1_pair && m6)
      LAUNCH_PE((k_dyn_cells1_p<6, false>), (k_dyn_cells1_p<6, true>), d.nCells, d, p, cf, s);
    else if (pair_layout(d) && g_cells1_pair)
      LAUNCH_PE((k_dyn_cells1_p<7, false>), (k_dyn_cells1_p<7, true>), d.nCells, d, p, cf, s);
    else if (m6) LAUNCH(k_dyn_cells1_b<6>, d.nCells, d, p, cf, s);
    else LAUNCH(k_dyn_cells1_b<7>, d.nCells, d, p, cf, s);
  }
  if (part == 1) return;
  if (pair_layout(d)) {
    const int64_t nw = d.nEdges;
    if (rk_step == 1) LAUNCH_PE((k_dyn_edges_pgf_p<false>), (k_dyn_edges_pgf_p<true>), nw, d, p);
    if (d.maxEdges == 6 && rk_step == 1) LAUNCH_PE((k_dyn_edges_p<true, 10, true, false>), (k_dyn_edges_p<true, 10, true, true>), nw, d, p, cf, s, 0);
    if (d.maxEdges == 6 && rk_step != 1) LAUNCH_PE((k_dyn_edges_p<false, 10, false, false>), (k_dyn_edges_p<false, 10, false, true>), nw, d, p, cf, s, 1, tp);
    if (d.maxEdges == 7 && rk_step == 1) LAUNCH_PE((k_dyn_edges_p<true, 12, true, false>), (k_dyn_edges_p<true, 12, true, true>), nw, d, p, cf, s, 0);
    if (d.maxEdges == 7 && rk_step != 1) LAUNCH_PE((k_dyn_edges_p<false, 12, false, false>), (k_dyn_edges_p<false, 12, false, true>), nw, d, p, cf, s, 1, tp);
  } else if (batched(d)) {
    if (d.maxEdges == 6 && rk_step == 1) LAUNCH_E((k_dyn_edges_b<true, 10>), d.nEdges, d, p, cf, s, 0);
    if (d.maxEdges == 6 && rk_step != 1) LAUNCH_E((k_dyn_edges_b<false, 10>), d.nEdges, d, p, cf, s, 1);
    if (d.maxEdges == 7 && rk_step == 1) LAUNCH_E((k_dyn_edges_b<true, 12>), d.nEdges, d, p, cf, s, 0);
    if (d.maxEdges == 7 && rk_step != 1) LAUNCH_E((k_dyn_edges_b<false, 12>), d.nEdges, d, p, cf, s, 1);
  } else if (rk_step == 1)
    LAUNCH(k_dyn_edges<true>, d.nEdges, d, p, cf, s, 0);
  else
    LAUNCH(k_dyn_edges<false>, d.nEdges, d, p, cf, s, 1);
  if (rk_step == 1) {
    if (!bt) {
      if (s.h_mom_eddy_visc4 > 0.0) LAUNCH(k_dyn_delsq_vc, d.nVertices + d.nCells, d, p);
      LAUNCH(k_dyn_edges_rk1b, d.nEdgesSolve, d, p, cf, s);
      LAUNCH(k_dyn_cells2, d.nCells, d, p);
    } else {
      if (s.h_mom_eddy_visc4 > 0.0) {
        if (pair_layout(d) && g_delsq_pair) {  // interleaved, PAIR_EPW elements per wavefront
          const int64_t nw = 3 * std::max<int64_t>((d.nVertices + 2 * PAIR_EPW - 1) / (2 * PAIR_EPW),
                                                   (d.nCells + PAIR_EPW - 1) / PAIR_EPW);
          if (m6) LAUNCH_PE((k_dyn_delsq_vc_p<6, false>), (k_dyn_delsq_vc_p<6, true>), nw * PAIR_EPW, d, p);
          else LAUNCH_PE((k_dyn_delsq_vc_p<7, false>), (k_dyn_delsq_vc_p<7, true>), nw * PAIR_EPW, d, p);
        } else {
          const int nvc = 3 * std::max((d.nVertices + 1) / 2, d.nCells);  // interleaved (k_dyn_delsq_vc_b)
          if (m6) LAUNCH(k_dyn_delsq_vc_b<6>, nvc, d, p);
          else LAUNCH(k_dyn_delsq_vc_b<7>, nvc, d, p);
        }
      }
      LAUNCH(k_dyn_edges_rk1b_b, d.nEdgesSolve, d, p, cf, s, tp);
      if (pair_layout(d) && g_cells2_pair) {
        if (m6) LAUNCH_PE((k_dyn_cells2_p<6, false>), (k_dyn_cells2_p<6, true>), d.nCells, d, p);
        else LAUNCH_PE((k_dyn_cells2_p<7, false>), (k_dyn_cells2_p<7, true>), d.nCells, d, p);
      } else if (m6) {
        LAUNCH(k_dyn_cells2_b<6>, d.nCells, d, p);
      } else {
        LAUNCH(k_dyn_cells2_b<7>, d.nCells, d, p);
      }
    }
  }
  if (!batched(d)) LAUNCH(k_dyn_advflux, d.nEdges, d, p);
  else if (pair_layout(d) && d.maxEdges == 6) LAUNCH_PE((k_dyn_advflux_p<10, false>), (k_dyn_advflux_p<10, true>), d.nEdges, d, p);
  else if (pair_layout(d)) LAUNCH_PE((k_dyn_advflux_p<12, false>), (k_dyn_advflux_p<12, true>), d.nEdges, d, p);
  else if (d.maxEdges == 6) LAUNCH_E(k_dyn_advflux_b<10>, d.nEdges, d, p);
  else LAUNCH_E(k_dyn_advflux_b<12>, d.nEdges, d, p);
  if (batched(d)) {
    const bool sml = fuse_smlstep(d);
    if (d.maxEdges == 6 && rk_step == 1 && sml) LAUNCH((k_dyn_cells3_r<6, true, true>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 6 && rk_step != 1 && sml) LAUNCH((k_dyn_cells3_r<6, false, true>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 7 && rk_step == 1 && sml) LAUNCH((k_dyn_cells3_r<7, true, true>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 7 && rk_step != 1 && sml) LAUNCH((k_dyn_cells3_r<7, false, true>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 6 && rk_step == 1 && !sml) LAUNCH((k_dyn_cells3_r<6, true>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 6 && rk_step != 1 && !sml) LAUNCH((k_dyn_cells3_r<6, false>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 7 && rk_step == 1 && !sml) LAUNCH((k_dyn_cells3_r<7, true>), d.nCellsSolve, d, p, cf, s);
    if (d.maxEdges == 7 && rk_step != 1 && !sml) LAUNCH((k_dyn_cells3_r<7, false>), d.nCellsSolve, d, p, cf, s);
    return;
  }
  LAUNCH(k_dyn_cells3, d.nCellsSolve, d, p, cf, s);
}

// tu_up: the block's fused-unpack map of the tend_u exchange (642), used by phase 2, or none
void smlstep_pert(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, int phase, XUnpack tu_up = XUnpack{}) {
  if (fuse_smlstep(d)) {  // k_dyn_cells3_r did the cells without a halo edge
    if (phase == 1) return;
    phase = 2;
  }
  const int64_t nb = phase == 2 ? d.n_bnd_cells : d.nCellsSolve;  // phase 2: the bnd_cells list
  if (!batched(d)) LAUNCH(k_smlstep_pert, d.nCellsSolve, d, p, phase);
  else if (d.maxEdges == 6) LAUNCH(k_smlstep_pert_b<6>, nb, d, p, phase, tu_up);
  else LAUNCH(k_smlstep_pert_b<7>, nb, d, p, phase, tu_up);
}

// hdiv = 1: the batched kernel also computes the next stage's h_divergence (k_recover_cells3_b)
void recover_cells3(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, int phase, int hdiv = 0) {
  if (!batched(d)) LAUNCH(k_recover_cells3, d.nCells, d, p, phase);
  else if (d.maxEdges == 6) LAUNCH(k_recover_cells3_b<6>, d.nCells, d, p, phase, hdiv);
  else LAUNCH(k_recover_cells3_b<7>, d.nCells, d, p, phase, hdiv);
}

double coef_divdamp(const mpas_dyc_ctx* ctx, double dts) {  // 2761-2763
  const double rdts = 1.0 / dts;
  return 2.0 * ctx->cf.smdiv * ctx->cf.len_disp * rdts;
}

// edge phase of acoustic sub-step `small_step`; damp = 1 also applies the divergence damping of
// the previous sub-step (k_acoustic_edges<true>); fresh = 1 when that sub-step was sub-step 1,
// whose edge phase is not launched (its ru_p = ruAvg = dts * tend_u are formed by the readers)
// um: the block's fused-unpack map of the exchange just completed (pair layout only), or none
void acoustic_edges(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, double dts, int small_step, int damp,
                    int phase, int fresh = 0, UnpackMap um = UnpackMap{}) {
  if (pair_layout(d)) {
    const int64_t nw = phase == 2 ? d.n_bnd_pairs : d.nEdges;  // phase 2: the bnd_pairs list
    const bool up = um.recv != nullptr;
    if (damp && up)
      LAUNCH_PE((k_acoustic_edges_p<true, true, false>), (k_acoustic_edges_p<true, true, true>), nw, d, p, dts, small_step, coef_divdamp(ctx, dts), phase, fresh, um);
    else if (damp)
      LAUNCH_PE((k_acoustic_edges_p<true, false, false>), (k_acoustic_edges_p<true, false, true>), nw, d, p, dts, small_step, coef_divdamp(ctx, dts), phase, fresh, um);
    else if (up)
      LAUNCH_PE((k_acoustic_edges_p<false, true, false>), (k_acoustic_edges_p<false, true, true>), nw, d, p, dts, small_step, 0.0, phase, fresh, um);
    else
      LAUNCH_PE((k_acoustic_edges_p<false, false, false>), (k_acoustic_edges_p<false, false, true>), nw, d, p, dts, small_step, 0.0, phase, fresh, um);
    return;
  }
  if (damp)
    LAUNCH_E(k_acoustic_edges<true>, d.nEdges, d, p, dts, small_step, coef_divdamp(ctx, dts), phase, fresh);
  else
    LAUNCH_E(k_acoustic_edges<false>, d.nEdges, d, p, dts, small_step, 0.0, phase, fresh);
}

// the record kernels fuse the owned cells' recover_cells1 into a stage's last sub-step
bool fused_recover(const Dims& d) { return batched(d) && (d.maxEdges == 6 || d.maxEdges == 7); }

// fin = 1: the stage's last sub-step, which also recovers the owned cells (k_acoustic_cells_r<ME,
// true>) when fused_recover(d); rdt / invNs / rk_step are k_recover_cells1's arguments
// keep_pp = 0: a fin launch need not store rho_pp / rw_p (see k_acoustic_cells_r)
// pk: the block's fused-pack map of the exchange that follows (fused_pack_map), or none
// dl: store rtheta_pp - rtheta_pp_old for the stage's last damping only (damping_delta)
// rp (fin only): the block's pack map of the 876-887 exchange that follows the stage (XPlan::fused_rec)
void acoustic_cells(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, double dts, int small_step, int fin = 0,
                    double rdt = 0.0, double invNs = 0.0, int rk_step = 0, int keep_pp = 1, PackMap pk = PackMap{},
                    int dl = 0, XPack rp = XPack{}) {
  if (batched(d) && d.maxEdges == 6) {
    if (fin)
      LAUNCH((k_acoustic_cells_r<6, true>), d.nCells, d, p, dts, small_step, ctx->cf.epssm, rdt, invNs, rk_step, keep_pp,
             pk, dl, rp);
    else LAUNCH((k_acoustic_cells_r<6, false>), d.nCells, d, p, dts, small_step, ctx->cf.epssm, 0.0, 0.0, 0, 1, pk);
    return;
  }
  if (batched(d) && d.maxEdges == 7) {
    if (fin)
      LAUNCH((k_acoustic_cells_r<7, true>), d.nCells, d, p, dts, small_step, ctx->cf.epssm, rdt, invNs, rk_step, keep_pp,
             pk, dl, rp);
    else LAUNCH((k_acoustic_cells_r<7, false>), d.nCells, d, p, dts, small_step, ctx->cf.epssm, 0.0, 0.0, 0, 1, pk);
    return;
  }
  LAUNCH(k_acoustic_cells, d.nCells, d, p, dts, small_step, ctx->cf.epssm);
}

// The stage's last cell phase hands its damping rtheta_pp - rtheta_pp_old instead of both
// fields when nothing else reads them before the next stage: no exchange (the 845 and 876-887
// exchanges and the halo-cell recovery read rtheta_pp) and not the dt's last stage (whose values
// the pool keeps); the fused cell recovery takes rtheta_pp from registers.  Pair-layout damping
// and record cell kernels only.
inline int damping_delta(const mpas_dyc_ctx* ctx, const Dims& d, bool last_stage) {
  return (!needs_exchange(ctx) && !last_stage && pair_layout(d) && fused_recover(d)) ? 1 : 0;
}

// the last damping of a stage also recovers the edges with two owned cells (k_divdamp_p<true>);
// needs the owned cells' rho_zz recovered by the last cell phase (fused_recover)
bool fused_recover_edges(const Dims& d) { return pair_layout(d) && fused_recover(d); }

// fresh = 1: the stage had a single sub-step (no edge phase launched), see k_divdamp_p;
// invNs > 0: recover the edges with two owned cells too (fused_recover_edges)
// dl: rtheta_pp_old holds the difference (acoustic_cells with dl); pair layout only
// rp: the block's pack map of the 876-887 exchange (XPlan::fused_rec), or none
// upk: the block's pack map of the u exchange (988, XPlan::fused_rec), used by the recovering variant
void divergence_damping(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, double dts, int phase, int fresh = 0,
                        double invNs = 0.0, UnpackMap um = UnpackMap{}, int dl = 0, XPack rp = XPack{},
                        XPack upk = XPack{}) {
  // (k_divdamp_b, one edge per wave with batched loads, measured 6 % slower than this)
  const bool up = um.recv != nullptr;
  const int64_t nw = phase == 2 ? d.n_bnd_pairs : d.nEdges;  // phase 2: the bnd_pairs list
  const double cd = coef_divdamp(ctx, dts);
  if (pair_layout(d) && invNs > 0.0 && fused_recover_edges(d)) {
    if (up) LAUNCH_PE((k_divdamp_p<true, true, false>), (k_divdamp_p<true, true, true>), nw, d, p, cd, phase, dts, fresh, invNs, um, dl, rp, upk);
    else LAUNCH_PE((k_divdamp_p<true, false, false>), (k_divdamp_p<true, false, true>), nw, d, p, cd, phase, dts, fresh, invNs, um, dl, rp, upk);
  } else if (pair_layout(d)) {
    if (up) LAUNCH_PE((k_divdamp_p<false, true, false>), (k_divdamp_p<false, true, true>), nw, d, p, cd, phase, dts, fresh, 0.0, um, dl, rp);
    else LAUNCH_PE((k_divdamp_p<false, false, false>), (k_divdamp_p<false, false, true>), nw, d, p, cd, phase, dts, fresh, 0.0, um, dl, rp);
  }
  else LAUNCH(k_divdamp<DIVDAMP_EPW>, (d.nEdges + DIVDAMP_EPW - 1) / DIVDAMP_EPW, d, p, coef_divdamp(ctx, dts), phase,
              dts, fresh);
}

// store_grad: gradPVt / gradPVn (5814-5815) are diag fields that nothing reads -- no routine of
// the dycore, and no later phase of this one (pv_edge uses the values in registers).  Every call
// overwrites them, so only the last call of a dt (and the model-init call) stores them: the pool
// holds the same values after the step, at 2 x 8 B per edge-level less traffic in 8 of 9 calls.
// uu_up: the block's fused-unpack map of the u exchange that precedes (988), or none
void solve_diagnostics(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, double dt, int tl, int rk_step /*0 = absent*/,
                       int store_grad = 1, XUnpack uu_up = XUnpack{}) {
  const double* u = (tl == 1) ? p.u1 : p.u2;
  const double* h = (tl == 1) ? p.rho_zz1 : p.rho_zz2;
  const int reconstruct_v = (rk_step == 0 || rk_step == 3) ? 1 : 0;
  // divergence and vorticity are read only by the rk1 dyn_tend (the del2 of u, 4856-4883): the
  // calls that precede an rk 2 / 3 stage need not store them (the pool keeps the dt's last values)
  const int store_dv = (rk_step == 0 || rk_step == 3) ? 1 : 0;
  if (!batched(d)) {
    LAUNCH(k_diag_vertices, d.nVertices, d, p, u, store_dv);
    LAUNCH(k_diag_cells, d.nCells, d, p, u, ctx->cf.apvm_upwinding, store_dv);
    LAUNCH(k_diag_edges, d.nEdges, d, p, u, h, reconstruct_v, ctx->cf.apvm_upwinding, dt, store_grad);
    return;
  }
  if (pair_layout(d)) {
    LAUNCH_PE((k_diag_vertices_p<false>), (k_diag_vertices_p<true>), d.nVertices, d, p, u, store_dv, uu_up,
              (tl == 1) ? p.u1 : p.u2);
    // (a pair-layout k_diag_cells, two cells per wave, measured 18 % slower than the batched one; a
    // round-5 version with the edge and vertex sums in two passes, 66 VGPRs, bitwise: 206 against
    // 202 us per call, profiles/r05_ab_diag_cells_pair_rejected.log)
    if (d.maxEdges == 6) LAUNCH(k_diag_cells_b<6>, d.nCells, d, p, u, ctx->cf.apvm_upwinding, store_dv);
    else LAUNCH(k_diag_cells_b<7>, d.nCells, d, p, u, ctx->cf.apvm_upwinding, store_dv);
    const int64_t nw = d.nEdges;
    if (d.maxEdges == 6) LAUNCH_PE((k_diag_edges_p<10, false>), (k_diag_edges_p<10, true>), nw, d, p, u, h, reconstruct_v, ctx->cf.apvm_upwinding, dt, store_grad);
    else LAUNCH_PE((k_diag_edges_p<12, false>), (k_diag_edges_p<12, true>), nw, d, p, u, h, reconstruct_v, ctx->cf.apvm_upwinding, dt, store_grad);
  } else if (d.maxEdges == 6) {
    LAUNCH(k_diag_vertices, d.nVertices, d, p, u, store_dv);  // (a batched one-column variant measured slower)
    LAUNCH(k_diag_cells_b<6>, d.nCells, d, p, u, ctx->cf.apvm_upwinding, store_dv);
    LAUNCH_E(k_diag_edges_b<10>, d.nEdges, d, p, u, h, reconstruct_v, ctx->cf.apvm_upwinding, dt, store_grad);
  } else {
    LAUNCH(k_diag_vertices, d.nVertices, d, p, u, store_dv);
    LAUNCH(k_diag_cells_b<7>, d.nCells, d, p, u, ctx->cf.apvm_upwinding, store_dv);
    LAUNCH_E(k_diag_edges_b<12>, d.nEdges, d, p, u, h, reconstruct_v, ctx->cf.apvm_upwinding, dt, store_grad);
  }
}

void advance_scalars(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, double dt, int rk_step, bool advance_density) {
  double wt_new = 1.0;
  if (advance_density) {
    if (rk_step == 1 && ctx->cf.time_integration_order == 3) wt_new = 1. / 3;
    if (rk_step == 1 && ctx->cf.time_integration_order == 2) wt_new = 1. / 2;
    if (rk_step == 2) wt_new = 1. / 2;
    if (rk_step == 3) wt_new = 1.;
  }
  if (batched(d) && pair_layout(d)) {
    if (d.maxEdges == 6 && d.ns == 1)
      LAUNCH_PE((k_scalars_edges_p<10, false, true>), (k_scalars_edges_p<10, true, true>), d.nEdges, d, p);
    else if (d.maxEdges == 6) LAUNCH_PE((k_scalars_edges_p<10, false>), (k_scalars_edges_p<10, true>), d.nEdges, d, p);
    else if (d.ns == 1) LAUNCH_PE((k_scalars_edges_p<12, false, true>), (k_scalars_edges_p<12, true, true>), d.nEdges, d, p);
    else LAUNCH_PE((k_scalars_edges_p<12, false>), (k_scalars_edges_p<12, true>), d.nEdges, d, p);
  } else {
    LAUNCH(k_scalars_edges, d.nEdges, d, p);
  }
  if (!batched(d)) LAUNCH(k_scalars_cells, d.nCellsSolve, d, p, dt, wt_new, ctx->cf.coef_3rd_order);
  else if (d.maxEdges == 6) LAUNCH(k_scalars_cells_b<6>, d.nCellsSolve, d, p, dt, wt_new, ctx->cf.coef_3rd_order);
  else LAUNCH(k_scalars_cells_b<7>, d.nCellsSolve, d, p, dt, wt_new, ctx->cf.coef_3rd_order);
}

// atm_advance_scalars_mono (3548-4210) over all blocks: its two halo exchanges
// (scalars_old at 3757, the limiter factors at 4098) sit between the block loops.
// the preparation (3737-3777: scalars_old += dt * tend / rho_zz_old, rho_zz_int) and its
// scalars_old exchange (3757); split out so srk3 can merge that exchange with the one before it
void mono_prep(mpas_dyc_ctx* ctx, const std::vector<Ptrs>& P, double dt, bool advance_density) {
  for (size_t b = 0; b < ctx->blk.size(); ++b) {
    const Dims& d = ctx->blk[b].d;
    if (!batched(d)) LAUNCH(k_mono_prep, d.nCells, d, P[b], dt, advance_density ? 1 : 0);
    else if (d.maxEdges == 6) LAUNCH(k_mono_prep_b<6>, d.nCells, d, P[b], dt, advance_density ? 1 : 0);
    else LAUNCH(k_mono_prep_b<7>, d.nCells, d, P[b], dt, advance_density ? 1 : 0);
  }
}

// The block's pointers with the monotone transport's per-scalar scratch (s_max, s_min, wdtn,
// flux_arr, flux_upwind_tmp, flux_tmp, scalar_old_copy, scale_arr) switched to its second set, which
// the second scalar of a pair uses
Ptrs mono_slot1(mpas_dyc_ctx* c, Block& b, Ptrs p) {
  p.s_max = P<double>(c, b, "scratch", "s_max_1");
  p.s_min = P<double>(c, b, "scratch", "s_min_1");
  p.scalar_old_copy = P<double>(c, b, "scratch", "scalar_old_copy_1");
  p.flux_arr = P<double>(c, b, "scratch", "flux_arr_1");
  p.flux_upwind_tmp = P<double>(c, b, "scratch", "flux_upwind_tmp_1");
  p.flux_tmp = P<double>(c, b, "scratch", "flux_tmp_1");
  p.scale_arr = P<double>(c, b, "scratch", "scale_arr_1");
  p.wdtn = P<double>(c, b, "scratch", "wdtn_1");
  return p;
}

// MPAS_DYCORE_MONO_PAIRS=0 (read when a context is created): one scalar at a time
int g_mono_pairs = 1;
// the monotone limiter's bounds (s_max, s_min, wdtn) inside the first cell pass k_mono_cells1_b<ME, true>
// (MPAS_DYCORE_MONO_FUSE=0, read when a context is created: the separate k_mono_bounds_b).  (The flux
// rescaling of k_mono_edges2_p inside k_mono_cells2_b, each edge formed by both of its cells, was bitwise
// but no faster: profiles/r05_ab_mono_fuse_edges2_rejected.log.)
constexpr int MONO_FUSE_BOUNDS = 1;
int g_mono_fuse = MONO_FUSE_BOUNDS;

// The reference's per-scalar loop (3798-4210): bounds, fluxes, limiter factors, the scale_arr
// exchange (4098), rescale and update, one scalar after the other.  Each scalar's pipeline reads and
// writes only its own scalar and its own scratch, so two scalars run it side by side here with two
// sets of scratch and one scale_arr exchange for both (half the exchanges, and half the RCCL groups
// between GPUs) -- the same operations on the same operands, bit for bit.
// prepared = true: mono_prep ran and its exchange was merged into the caller's
int advance_scalars_mono(mpas_dyc_ctx* ctx, const std::vector<Ptrs>& P, double dt, bool advance_density,
                         bool prepared = false) {
  const int ad = advance_density ? 1 : 0;
  const int nb = (int)ctx->blk.size();
  if (!prepared) {
    mono_prep(ctx, P, dt, advance_density);
    CHK(exchange(ctx, {{"state", "scalars", 1, ALL_LAYERS}}));
  }
  const int ns = ctx->blk[0].d.ns;
  std::vector<Ptrs> P1;
  if (ns >= 2 && g_mono_pairs)
    for (int b = 0; b < nb; ++b) P1.push_back(mono_slot1(ctx, ctx->blk[b], P[b]));
  for (int is = 0; is < ns; is += (P1.empty() ? 1 : 2)) {
    const int nq = (!P1.empty() && is + 1 < ns) ? 2 : 1;  // scalars in this pass
    for (int b = 0; b < nb; ++b) {
      const Dims& d = ctx->blk[b].d;
      const bool bt = batched(d), m6 = d.maxEdges == 6;
      // the pair's second scratch set for the kernels that take both scalars in one launch
      const MonoCell2 s2 = nq == 2 ? MonoCell2{P1[b].wdtn, P1[b].s_max, P1[b].s_min, P1[b].flux_arr,
                                               P1[b].flux_upwind_tmp, P1[b].scalar_old_copy, P1[b].scale_arr}
                                   : MonoCell2{};
      const double c3 = ctx->cf.coef_3rd_order;
      const bool fb = bt && (g_mono_fuse & MONO_FUSE_BOUNDS);  // the bounds inside k_mono_cells1_b<ME, true>
      if (!bt) {
        for (int q = 0; q < nq; ++q) LAUNCH(k_mono_bounds, d.nCellsSolve, d, q ? P1[b] : P[b], is + q, c3);
      } else if (fb) {
      } else if (m6) {
        LAUNCH(k_mono_bounds_b<6>, d.nCellsSolve, d, P[b], is, c3, nq, s2);
      } else {
        LAUNCH(k_mono_bounds_b<7>, d.nCellsSolve, d, P[b], is, c3, nq, s2);
      }
      if (batched(d) && pair_layout(d)) {  // both scalars of the pair in one launch (the rows read once)
        const MonoFlux2 f2 = nq == 2 ? MonoFlux2{P1[b].flux_arr, P1[b].flux_upwind_tmp, P1[b].flux_tmp} : MonoFlux2{};
        if (m6) LAUNCH_PE((k_mono_edges1_p<10, false>), (k_mono_edges1_p<10, true>), d.nEdges, d, P[b], is, dt, nq, f2);
        else LAUNCH_PE((k_mono_edges1_p<12, false>), (k_mono_edges1_p<12, true>), d.nEdges, d, P[b], is, dt, nq, f2);
      } else {
        for (int q = 0; q < nq; ++q) LAUNCH(k_mono_edges1, d.nEdges, d, q ? P1[b] : P[b], is + q, dt);
      }
      if (bt) {  // both scalars of the pair in one launch (the cell's own columns read once)
        const int pr = pair_layout(d) ? 1 : 0;  // which edge kernel formed the fluxes
        if (fb && m6) LAUNCH((k_mono_cells1_b<6, true>), d.nCellsSolve, d, P[b], is, dt, ad, nq, s2, pr, c3);
        else if (fb) LAUNCH((k_mono_cells1_b<7, true>), d.nCellsSolve, d, P[b], is, dt, ad, nq, s2, pr, c3);
        else if (m6) LAUNCH(k_mono_cells1_b<6>, d.nCellsSolve, d, P[b], is, dt, ad, nq, s2, pr);
        else LAUNCH(k_mono_cells1_b<7>, d.nCellsSolve, d, P[b], is, dt, ad, nq, s2, pr);
      } else {
        for (int q = 0; q < nq; ++q) LAUNCH(k_mono_cells1, d.nCellsSolve, d, q ? P1[b] : P[b], is + q, dt, ad);
      }
    }
    if (nq == 2) CHK(exchange(ctx, {{"scratch", "scale_arr", 1, 0x1u}, {"scratch", "scale_arr_1", 1, 0x1u}}));
    else CHK(exchange(ctx, {{"scratch", "scale_arr", 1, 0x1u}}));
    for (int b = 0; b < nb; ++b) {
      const Dims& d = ctx->blk[b].d;
      if (!batched(d)) {
        for (int q = 0; q < nq; ++q) {
          const Ptrs& pq = q ? P1[b] : P[b];
          LAUNCH(k_mono_edges2, d.nEdges, d, pq, dt);
          LAUNCH(k_mono_cells2, d.nCells, d, pq, is + q, ad);
        }
        continue;
      }
      // each scalar's edge pass, then both scalars' cell pass in one launch (each scalar's pipeline
      // touches only its own scalar and scratch set: the order between the two does not matter)
      for (int q = 0; q < nq; ++q) {
        const Ptrs& pq = q ? P1[b] : P[b];
        if (pair_layout(d)) LAUNCH_PE((k_mono_edges2_p<false>), (k_mono_edges2_p<true>), d.nEdges, d, pq, dt);
        else LAUNCH(k_mono_edges2, d.nEdges, d, pq, dt);
      }
      const MonoCell2 s2 = nq == 2 ? MonoCell2{P1[b].wdtn, P1[b].s_max, P1[b].s_min, P1[b].flux_arr,
                                               P1[b].flux_upwind_tmp, P1[b].scalar_old_copy, P1[b].scale_arr}
                                   : MonoCell2{};
      double* fa2 = nq == 2 ? P1[b].flux_arr : nullptr;
      if (d.maxEdges == 6) LAUNCH(k_mono_cells2_b<6>, d.nCells, d, P[b], is, ad, nq, s2, fa2);
      else LAUNCH(k_mono_cells2_b<7>, d.nCells, d, P[b], is, ad, nq, s2, fa2);
    }
  }
  return MPAS_DYC_OK;
}

std::vector<Ptrs> block_ptrs(mpas_dyc_ctx* ctx) {
  std::vector<Ptrs> P;
  for (auto& b : ctx->blk) P.push_back(make_ptrs(ctx, b));
  return P;
}

// summarize_timestep (1794 -> 6675-7018): the fields its enabled modes reduce, on time level
// `tl` of block b.  0 = w, 1 = u (with v for the wind speed in detailed mode), 2.. = scalars.
std::vector<SumField> summary_fields(mpas_dyc_ctx* ctx, Block& b, int tl) {
  const Dims& d = b.d;
  const int fl = ctx->summary_flags;
  std::vector<SumField> fs;
  const bool vel = fl & (MPAS_DYC_PRINT_GLOBAL_MINMAX_VEL | MPAS_DYC_PRINT_DETAILED_MINMAX_VEL);
  const bool det = fl & MPAS_DYC_PRINT_DETAILED_MINMAX_VEL;
  SumField w{}, u{};
  w.a = P<const double>(ctx, b, "state", "w", tl);
  w.ncol = vel ? d.nCellsSolve : 0;
  w.K = d.K;
  w.stride = d.K + 1;
  u.a = P<const double>(ctx, b, "state", "u", tl);
  u.ncol = vel ? d.nEdgesSolve : 0;
  u.K = d.K;
  u.stride = d.K;
  if (det) {
    w.lat = P<const double>(ctx, b, "mesh", "latCell");
    w.lon = P<const double>(ctx, b, "mesh", "lonCell");
    u.v = P<const double>(ctx, b, "diag", "v");
    u.lat = P<const double>(ctx, b, "mesh", "latEdge");
    u.lon = P<const double>(ctx, b, "mesh", "lonEdge");
  }
  fs.push_back(w);
  fs.push_back(u);
  const double* sc = P<const double>(ctx, b, "state", "scalars", tl);
  for (int is = 0; is < d.ns; ++is) {
    SumField s{};
    s.a = sc + (size_t)is * (d.nCells + 1) * d.K;  // scalar-major [ns][nCells+1][K]
    s.ncol = (fl & MPAS_DYC_PRINT_GLOBAL_MINMAX_SCA) ? d.nCellsSolve : 0;
    s.K = d.K;
    s.stride = d.K;
    fs.push_back(s);
  }
  return fs;
}

// the device half of summarize_timestep: per-block records in Block::sum_out (mpas_dyc_get_summary
// folds blocks and ranks)
int summary_launch(mpas_dyc_ctx* ctx, int tl) {
  if (!ctx->summary_flags || ctx->planning) return MPAS_DYC_OK;
  for (auto& b : ctx->blk) {
    const std::vector<SumField> fs = summary_fields(ctx, b, tl);
    for (size_t f0 = 0; f0 < fs.size(); f0 += SUM_MAX_FIELDS) {
      const int nf = (int)std::min<size_t>(SUM_MAX_FIELDS, fs.size() - f0);
      SumFields sf{};
      for (int i = 0; i < nf; ++i) sf.f[i] = fs[f0 + i];
      hipLaunchKernelGGL(k_summary_partial, dim3(SUM_PARTS, nf), dim3(256), 0, ctx->stream, sf, b.sum_part);
      hipLaunchKernelGGL(k_summary_final, dim3(nf), dim3(256), 0, ctx->stream, sf, b.sum_part, SUM_PARTS,
                         b.sum_out + f0 * SUM_REC);
    }
  }
  ctx->summary_tl = tl;
  return MPAS_DYC_OK;
}

// run `body(d, p)` for every block (the reference's `block => domain % blocklist` loops), with the
// blocks' pointers from the vector V (EACH: P)
#define EACHV(V, ...)                                   \
  for (size_t ib_ = 0; ib_ < ctx->blk.size(); ++ib_) {  \
    const Dims& d = ctx->blk[ib_].d;                    \
    const Ptrs& p = (V)[ib_];                           \
    (void)d;                                            \
    (void)p;                                            \
    __VA_ARGS__;                                        \
  }
#define EACH(...) EACHV(P, __VA_ARGS__)

// mpas_reconstruct (operators/mpas_vector_reconstruction.F:195-294): the cell-centre velocity
void reconstruct(mpas_dyc_ctx* ctx, const Dims& d, const Ptrs& p, const double* u) {
  if (batched(d) && d.maxEdges == 6) LAUNCH(k_reconstruct_b<6>, d.nCellsSolve, d, p, u);
  else if (batched(d)) LAUNCH(k_reconstruct_b<7>, d.nCellsSolve, d, p, u);
  else LAUNCH(k_reconstruct, d.nCellsSolve, d, p, u);
}

// atm_srk3 (mpas_atm_time_integration.F:142-1796)
// atm_bdy_adjust_scalars (6436-6586) at the end of a transport stage: the scalars' halo first
// (the filter reads the neighbours), then the relaxation / specified-zone update of owned cells
int lbc_scalars(mpas_dyc_ctx* ctx, const std::vector<Ptrs>& P, double dt, double dt_rk) {
  CHK(exchange(ctx, {{"state", "scalars", 2, ALL_LAYERS}}));
  EACH(LAUNCH(k_lbc_scalars_tmp, d.nCellsSolve, d, p, dt, dt_rk, dt_rk));
  EACH(LAUNCH(k_lbc_scalars_copy, d.nCellsSolve, d, p));
  return MPAS_DYC_OK;
}

// The end of atm_srk3 after the microphysics (1650-1660): the regional reset of the specified
// zone, "because microphysics has messed with them" (1672-1790), then summarize_timestep (1794) --
// its reductions on the device, the log lines on the host.
int step_tail(mpas_dyc_ctx* ctx, const std::vector<Ptrs>& P, double dt) {
  if (ctx->lbc) {
    EACH(LAUNCH(k_lbc_reset_spec, d.nCellsSolve, d, p, dt));       // 1672-1711
    CHK(exchange(ctx, {{"state", "scalars", 2, ALL_LAYERS}}));       // 1714-1790
    EACH(LAUNCH(k_lbc_set_scalars, d.nCellsSolve, d, p, dt));
  }
  return summary_launch(ctx, 2);
}

int srk3(mpas_dyc_ctx* ctx, double dt) {
  const Config& cf = ctx->cf;
  // P: the fields; Ppre / Pfin: what a dynamics substep's first stage reads before its recovery
  // (stage_pre, stage_fin), rebuilt after every rotation of the buffers
  std::vector<Ptrs> P = block_ptrs(ctx), Ppre, Pfin;
  auto relayout = [&](bool first_substep) {
    P = block_ptrs(ctx);
    Ppre.clear();
    Pfin.clear();
    for (const Ptrs& q : P) {
      Ppre.push_back(stage_pre(q, first_substep));
      Pfin.push_back(stage_fin(q, first_substep));
    }
  };
  int dynamics_split = cf.dynamics_split_steps;
  double dt_dynamics;
  if (cf.split_dynamics_transport) {
    dt_dynamics = dt / (double)dynamics_split;
  } else {
    dynamics_split = 1;
    dt_dynamics = dt;
  }
  const int nss = cf.number_of_sub_steps;
  double rk_timestep[3], rk_sub_timestep[3];
  int number_sub_steps[3];
  if (cf.time_integration_order == 3) {
    rk_timestep[0] = dt_dynamics / 3.;
    rk_timestep[1] = dt_dynamics / 2.;
    rk_timestep[2] = dt_dynamics;
    rk_sub_timestep[0] = dt_dynamics / 3.;
    rk_sub_timestep[1] = dt_dynamics / (double)nss;
    rk_sub_timestep[2] = dt_dynamics / (double)nss;
    number_sub_steps[0] = 1;
    number_sub_steps[1] = std::max(1, nss / 2);
    number_sub_steps[2] = nss;
  } else {
    rk_timestep[0] = dt_dynamics / 2.;
    rk_timestep[1] = dt_dynamics / 2.;
    rk_timestep[2] = dt_dynamics;
    rk_sub_timestep[0] = dt_dynamics / (double)nss;
    rk_sub_timestep[1] = dt_dynamics / (double)nss;
    rk_sub_timestep[2] = dt_dynamics / (double)nss;
    number_sub_steps[0] = std::max(1, nss / 2);
    number_sub_steps[1] = std::max(1, nss / 2);
    number_sub_steps[2] = nss;
  }
  const bool scalars_in_dynamics = cf.scalar_advection && !cf.split_dynamics_transport;
  const bool split = split_phase(ctx);
  const bool lbc = ctx->lbc;  // config_apply_lbcs: regional boundary updates at the reference's points
  // 329-338, plus the exner exchange of the first dynamics substep (513): nothing writes exner
  // in between (vert_imp_coefs reads it on owned cells only), so the halo values are the same
  CHK(exchange(ctx, {{"state", "theta_m", 1, ALL_LAYERS}, {"state", "scalars", 1, ALL_LAYERS},
                     {"diag", "pressure_p", 0, ALL_LAYERS}, {"diag", "rtheta_p", 0, ALL_LAYERS},
                     {"diag", "exner", 0, ALL_LAYERS}}));
  rotate_saves(ctx);                                              // 341-381: the saves,
  relayout(true);                                                 // time level 2 via stage_pre
  EACH(rk_integration_setup(ctx, d, p));
  EACH(LAUNCH(k_moist_cells, d.nCells, d, p));                    // 383-422
  EACH(if (pair_layout(d)) LAUNCH_PE((k_moist_edges_p<false>), (k_moist_edges_p<true>), d.nEdges, d, p);
       else LAUNCH(k_moist_edges, d.nEdges, d, p));
  // physics tendencies are zero without DO_PHYSICS (450-457): scratch arrays stay zero.

  // Deferred exchanges.  With split-phase exchanges, the exchange after the diagnostics
  // (1234-1249) runs on the exchange stream while the next kernels that do not read its fields
  // run: the next stage's k_dyn_cells1, and vert_imp_coefs where it comes first.  Without
  // split-phase exchanges, xchg blocks and xwait is a no-op, and the launch order is the same.
  auto xchg = [&](const std::vector<XField>& fs) { return split ? exchange_async(ctx, fs) : (exchange)(ctx, fs); };
  auto xwait = [&]() { return split ? exchange_wait(ctx) : MPAS_DYC_OK; };
  bool pending = false;  // an xchg whose xwait is still due
  bool final_pending = false;  // the last substep's 1234-1249 exchange, waited for after substep_finish
  // The w recovery of a stage computes the next stage's h_divergence (k_recover_cells3_b with hdiv),
  // so that stage's k_dyn_cells1 (which computes nothing else at rk 2 / 3) is not launched.  Without
  // split-phase exchanges: after stages 1 and 2.  With them, k_dyn_cells1 is the work that overlaps
  // the 1234-1249 exchange; at rk 2 of order 3 vert_imp_coefs overlaps it as well, so the fusion is
  // kept after stage 1 only.  Not with LBCs (the reference recomputes h_divergence from the
  // overwritten ru).
  bool hdiv_prev = false;  // the previous stage's w recovery computed this stage's h_divergence
  // split-phase exchanges that would have work to overlap: 642 when smlstep_pert is not fused into
  // k_dyn_cells3_r on some block, 876-887 when some block recovers its owned elements separately
  bool sml_fused = true, rec_overlap = false;
  for (const auto& b : ctx->blk) {
    sml_fused = sml_fused && fuse_smlstep(b.d);
    rec_overlap = rec_overlap || !fused_recover(b.d) || !fused_recover_edges(b.d);
  }
  if (ctx->overlap_all) sml_fused = false, rec_overlap = true;
  EACHV(Ppre, vert_imp_coefs(ctx, d, p, rk_sub_timestep[0]));    // 476-510 of dynamics substep 1
  for (int dynamics_substep = 1; dynamics_substep <= dynamics_split; ++dynamics_substep) {
    // 513 (exner): carried by the step-start exchange and by the 1282-1297 exchange below
    for (int rk_step = 1; rk_step <= 3; ++rk_step) {
      if (cf.time_integration_order == 3 && rk_step == 2) EACH(vert_imp_coefs(ctx, d, p, rk_sub_timestep[1]));
      const bool last_stage = dynamics_substep == dynamics_split && rk_step == 3;
      const bool hdiv_next = !lbc && rk_step < 3 && (!split || (rk_step == 1 && cf.time_integration_order == 3));
      // the first stage reads time level 2 and the saved fields through stage_pre until its recovery
      const std::vector<Ptrs>& PS = rk_step == 1 ? Ppre : P;
      const std::vector<Ptrs>& PF = rk_step == 1 ? Pfin : P;  // the stage's last cell phase
      // the tend_u exchange (642) packed by the final tend_u kernel and unpacked by smlstep_pert
      // (XPlan::fused_rec), or nullptr
      const std::vector<XField> xtu = {{"tend", "u", 0, 0x1u}};
      const XPlan* xt = fused_rec_plan(ctx, xtu);
      auto tpk = [&](size_t ib) { return xt ? xt->rpk_edge[ib] : XPack{}; };
      auto tup = [&](size_t ib) { return xt ? xt->rup_edge[ib] : XUnpack{}; };
      if (pending) {  // 561-630, k_dyn_cells1 overlapping the exchange
        EACHV(PS, dyn_tend(ctx, d, p, rk_step, dt, 1, hdiv_prev && batched(d)));
        CHK(xwait());
        pending = false;
        EACHV(PS, dyn_tend(ctx, d, p, rk_step, dt, 2, false, last_stage, tpk(ib_)));
      } else {
        EACHV(PS, dyn_tend(ctx, d, p, rk_step, dt, 0, hdiv_prev && batched(d), last_stage, tpk(ib_)));  // 561-630
      }
      const double dts = rk_sub_timestep[rk_step - 1];
      if (split && !sml_fused) {  // 642 | 644-678: interior cells overlap the tend_u exchange
        CHK(exchange_async(ctx, xtu));
        EACHV(PS, smlstep_pert(ctx, d, p, 1));
        CHK(exchange_wait(ctx));
        EACHV(PS, smlstep_pert(ctx, d, p, 2, tup(ib_)));
      } else if (split) {
        // k_dyn_cells3_r already did the interior cells' smlstep: nothing would overlap the exchange,
        // so it blocks (a fork and a join of the exchange stream cost more than they could hide)
        CHK(exchange(ctx, xtu));
        EACHV(PS, smlstep_pert(ctx, d, p, 2, tup(ib_)));
      } else {
        CHK(exchange(ctx, xtu));                                  // 642
        EACHV(PS, smlstep_pert(ctx, d, p, 0, tup(ib_)));          // 644-678
      }
      if (lbc) {  // 683-778: specified-zone tendencies, then the relaxation zone toward the driving state
        const double tds = dt_dynamics * (double)(dynamics_substep - 1) + rk_timestep[rk_step - 1];
        EACHV(PS, LAUNCH(k_lbc_spec_tend_cells, d.nCellsSolve, d, p));
        EACHV(PS, LAUNCH(k_lbc_spec_tend_edges, d.nEdgesSolve, d, p));
        EACHV(PS, LAUNCH(k_lbc_relax_cells, d.nCellsSolve, d, p, dt, tds));
        EACHV(PS, LAUNCH(k_lbc_relax_edges, d.nEdges, d, p, dt, tds));
      }
      // Acoustic sub-steps (788-870).
      // * Exchanges.  The reference exchanges rho_pp before every sub-step (792) and rtheta_pp
      //   after it (845).  Here the rho_pp exchange of sub-step n+1 travels with the rtheta_pp
      //   exchange of sub-step n.  Divergence damping, which runs in between, does not touch
      //   rho_pp, so the halo values are the same.  The exchange before sub-step 1 is dropped:
      //   that sub-step's edge phase does not read rho_pp (2580-2599), the cell phase reads and
      //   zeroes only owned columns (2617-2622), and the all-layer exchange at 876 overwrites
      //   those halo values before anything reads them.
      // * Damping.  The divergence damping of sub-step n (849-869) is fused into the edge phase
      //   of sub-step n+1 (k_acoustic_edges<true>).  Only the last sub-step's damping is a
      //   kernel of its own.
      // * Sub-step 1's edge phase (794-837 with small_step = 1) only sets ru_p = ruAvg =
      //   dts * tend_u on the edges with an owned cell.  It is not launched: its three readers
      //   form that product themselves -- the cell phase of sub-step 1, then either the damped
      //   edge phase of sub-step 2 or, for a one-sub-step stage, the damping, which also stores
      //   ruAvg (on the same edges, so the 876 exchange and the recovery see the same values).
      const int nsub = number_sub_steps[rk_step - 1];
      const std::vector<XField> xrec = {{"diag", "rw_p", 0, ALL_LAYERS}, {"diag", "ru_p", 0, ALL_LAYERS},  // 876-887
                                        {"diag", "rho_pp", 0, ALL_LAYERS}, {"diag", "rtheta_pp", 0, 0x2u}};
      // the 876-887 exchange packed by the stage's last cell phase and damping and unpacked by the
      // halo recovery (XPlan::fused_rec), or nullptr
      const XPlan* xr = fused_rec_plan(ctx, xrec);
      auto rpc = [&](size_t ib) { return xr ? xr->rpk_cell[ib] : XPack{}; };
      auto rpe = [&](size_t ib) { return xr ? xr->rpk_edge[ib] : XPack{}; };
      auto ruc = [&](size_t ib) { return xr ? xr->rup_cell[ib] : XUnpack{}; };
      auto rue = [&](size_t ib) { return xr ? xr->rup_edge[ib] : XUnpack{}; };
      // the u exchange after the recovery (988) packed where the recovery computes u and unpacked by
      // the diagnostics' vertex kernel (XPlan::fused_rec), or nullptr
      const std::vector<XField> xu = {{"state", "u", 2, ALL_LAYERS}};
      const XPlan* xuu = fused_rec_plan(ctx, xu);
      auto upk = [&](size_t ib) { return xuu ? xuu->rpk_edge[ib] : XPack{}; };
      auto uup = [&](size_t ib) { return xuu ? xuu->rup_edge[ib] : XUnpack{}; };
      // the last Theta''/rho'' exchange whose unpack its consumer does (XPlan::fused_unpack): the
      // next edge phase, or the stage's last damping
      const XPlan* unpack_xp = nullptr;
      auto um_of = [&](size_t ib) { return unpack_xp ? unpack_xp->unpack[ib] : UnpackMap{}; };
      for (int small_step = 1; small_step <= nsub; ++small_step) {
        if (small_step == 1) {
          // 794-837: formed by the readers (above)
        } else if (split) {  // interior edges overlap the exchange issued after the last cell phase
          EACHV(PS, acoustic_edges(ctx, d, p, dts, small_step, 1, 1, small_step == 2));
          CHK(exchange_wait(ctx));
          EACHV(PS, acoustic_edges(ctx, d, p, dts, small_step, 1, 2, small_step == 2, um_of(ib_)));
        } else {
          EACHV(PS, acoustic_edges(ctx, d, p, dts, small_step, 1, 0, small_step == 2, um_of(ib_)));
        }
        unpack_xp = nullptr;
        std::vector<XField> xf = {{"diag", "rtheta_pp", 0, 0x1u}};  // 845
        if (small_step < nsub) xf.push_back({"diag", "rho_pp", 0, 0x1u});  // 792 of the next sub-step
        const XPlan* xp = fused_pack_plan(ctx, xf);  // the cell phase packs this exchange's send buffer
        EACHV(small_step == nsub ? PF : PS,
              acoustic_cells(ctx, d, p, dts, small_step, small_step == nsub, rk_timestep[rk_step - 1],
                            1 / (double)nsub, rk_step, needs_exchange(ctx) || last_stage,
                            xp ? xp->pack[ib_] : PackMap{}, damping_delta(ctx, d, last_stage),
                            small_step == nsub ? rpc(ib_) : XPack{}));
        if (split) {
          CHK(exchange_async(ctx, xf));
        } else {
          CHK((exchange)(ctx, xf));  // parenthesised: no ADL lookup of std::exchange
        }
        if (xp && xp->fused_unpack) unpack_xp = xp;
      }
      if (split) {  // the last sub-step's damping (849-869), interior edges overlapping the exchange
        EACH(divergence_damping(ctx, d, p, dts, 1, nsub == 1, 1 / (double)nsub, UnpackMap{}, 0, rpe(ib_), upk(ib_)));
        CHK(exchange_wait(ctx));
        EACH(divergence_damping(ctx, d, p, dts, 2, nsub == 1, 0.0, um_of(ib_), 0, rpe(ib_)));
      } else {
        EACH(divergence_damping(ctx, d, p, dts, 0, nsub == 1, 1 / (double)nsub, um_of(ib_),
                                damping_delta(ctx, d, last_stage), rpe(ib_), upk(ib_)));
      }
      const double invNs = 1 / (double)number_sub_steps[rk_step - 1];
      const double rdt = rk_timestep[rk_step - 1];
      if (split) {
        // 889-1185: owned cells and interior edges overlap the 876-887 exchange; once every
        // owned u is final, the u exchange (988) overlaps the w recovery, which does not read u.
        // When the last cell phase and damping recovered those already (fused_recover,
        // fused_recover_edges) nothing is left to overlap and the exchange blocks.
        if (rec_overlap) CHK(exchange_async(ctx, xrec));
        else CHK((exchange)(ctx, xrec));
        // owned cells: recovered by the last sub-step's cell phase (fused_recover) or here
        EACH(if (!fused_recover(d)) LAUNCH(k_recover_cells1, d.nCells + 1, d, p, rdt, invNs, rk_step, 1, 0));
        // edges with two owned cells: recovered by the last damping (fused_recover_edges) or here
        EACH(if (!fused_recover_edges(d)) LAUNCH(k_recover_edges, d.nEdges, d, p, invNs, 1, XUnpack{}, upk(ib_)));
        if (rec_overlap) CHK(exchange_wait(ctx));
        EACH(LAUNCH(k_recover_cells1, d.nCells + 1 - d.nCellsSolve, d, p, rdt, invNs, rk_step, 2, d.nCellsSolve,
                    ruc(ib_)));
        EACH(LAUNCH(k_recover_edges, d.n_bnd_edges, d, p, invNs, 2, rue(ib_), upk(ib_)));  // phase 2: bnd_edges
        if (lbc) {  // the w recovery reads ru before the specified-zone overwrite (934-987)
          EACH(recover_cells3(ctx, d, p, 0));
          EACH(LAUNCH(k_lbc_u, d.nEdges, d, p, dt_dynamics * (double)(dynamics_substep - 1) + rk_timestep[rk_step - 1]));
          CHK(exchange(ctx, {{"state", "u", 2, ALL_LAYERS}}));  // 988
        } else {
          CHK(exchange_async(ctx, {{"state", "u", 2, ALL_LAYERS}}));
          EACH(recover_cells3(ctx, d, p, 0, hdiv_next));
          CHK(exchange_wait(ctx));
        }
      } else {
        // (The w recovery of the owned cells away from the halo before this exchange, straight after
        // the damping that recovered their edges' ru, and the rest after it: bitwise, but 2.5 % slower
        // per dt on the 8-way emulation -- profiles/r05_ab_early_w_rejected.log.)
        CHK((exchange)(ctx, xrec));
        // 889-930: the owned cells were recovered by the last sub-step if fused_recover
        EACH(if (fused_recover(d)) LAUNCH(k_recover_cells1, d.nCells + 1 - d.nCellsSolve, d, p, rdt, invNs, rk_step, 2,
                                          d.nCellsSolve, ruc(ib_));
             else LAUNCH(k_recover_cells1, d.nCells + 1, d, p, rdt, invNs, rk_step, 0, 0, ruc(ib_)));
        // the edges with two owned cells were recovered by the last damping if fused_recover_edges
        EACH(if (!fused_recover_edges(d)) LAUNCH(k_recover_edges, d.nEdges, d, p, invNs, 0, rue(ib_), upk(ib_));
             else LAUNCH(k_recover_edges, d.n_bnd_edges, d, p, invNs, 2, rue(ib_), upk(ib_)));
        // stages 1 and 2: also the next stage's h_divergence (dyn_tend then skips k_dyn_cells1)
        EACH(recover_cells3(ctx, d, p, 0, hdiv_next));
        if (lbc)  // 934-987
          EACH(LAUNCH(k_lbc_u, d.nEdges, d, p, dt_dynamics * (double)(dynamics_substep - 1) + rk_timestep[rk_step - 1]));
        CHK(exchange(ctx, {{"state", "u", 2, ALL_LAYERS}}));      // 988
      }
      if (scalars_in_dynamics) {                                  // 993-1185
        if (rk_step < 3 || (!cf.monotonic && !cf.positive_definite)) {
          EACH(advance_scalars(ctx, d, p, rk_timestep[rk_step - 1], rk_step, false));
        } else {
          CHK(advance_scalars_mono(ctx, P, rk_timestep[rk_step - 1], false));
        }
        if (lbc) CHK(lbc_scalars(ctx, P, dt, rk_timestep[rk_step - 1]));  // 1109-1180
      }
      EACH(solve_diagnostics(ctx, d, p, dt, 2, rk_step,             // 1187-1228
                             dynamics_substep == dynamics_split && rk_step == 3, uup(ib_)));
      std::vector<XField> xd = {{"state", "w", 2, ALL_LAYERS}, {"diag", "pv_edge", 0, ALL_LAYERS},  // 1234-1249
                                {"diag", "rho_edge", 0, ALL_LAYERS}};
      if (scalars_in_dynamics) xd.push_back({"state", "scalars", 2, ALL_LAYERS});
      if (lbc) {
        // regional: 1234-1249, the zero-gradient w of the specified zone and its exchange (1253-1270),
        // then (end of a dynamics substep) 1282-1297 -- blocking, in the reference's order
        CHK((exchange)(ctx, xd));
        EACH(LAUNCH(k_lbc_zero_grad_w, d.nCellsSolve, d, p));
        CHK((exchange)(ctx, {{"state", "w", 2, ALL_LAYERS}}));
        if (rk_step == 3 && dynamics_substep < dynamics_split) {
          CHK((exchange)(ctx, {{"state", "theta_m", 2, ALL_LAYERS}, {"diag", "pressure_p", 0, ALL_LAYERS},
                               {"diag", "rtheta_p", 0, ALL_LAYERS}, {"diag", "exner", 0, ALL_LAYERS}}));
          EACH(vert_imp_coefs(ctx, d, p, rk_sub_timestep[0]));     // 476-510 of the next substep
        }
      } else if (rk_step < 3) {
        CHK(xchg(xd));  // waited for inside the next stage's dyn_tend
        pending = true;
      } else if (dynamics_substep < dynamics_split) {
        // 1282-1297 follows 1234-1249 with nothing in between: one exchange carries both
        // (plus the next substep's 513, exner).  The next substep's vert_imp_coefs overlaps it:
        // it reads none of these fields' halos, and substep_finish, which now runs after it,
        // writes nothing it reads.
        xd.insert(xd.end(), {{"state", "theta_m", 2, ALL_LAYERS}, {"diag", "pressure_p", 0, ALL_LAYERS},
                             {"diag", "rtheta_p", 0, ALL_LAYERS}, {"diag", "exner", 0, ALL_LAYERS}});
        CHK(xchg(xd));
        EACH(vert_imp_coefs(ctx, d, p, rk_sub_timestep[0]));     // 476-510 of the next substep
        CHK(xwait());
      } else if (split) {
        // the dt's last 1234-1249: overlaps substep_finish, which reads and writes none of its
        // fields (w, pv_edge, rho_edge, scalars)
        CHK(exchange_async(ctx, xd));
        final_pending = true;
      } else {
        CHK((exchange)(ctx, xd));
      }
      hdiv_prev = hdiv_next;
    }
    if (!ctx->planning)                                           // 1304-1341
      EACH(hipLaunchKernelGGL(k_substep_finish_v, dim3(2048), dim3(BLOCK_THREADS), 0, ctx->stream, d, p,
                              dynamics_substep, dynamics_split, 1.0 / (double)dynamics_split));
    if (dynamics_substep < dynamics_split) {  // the saves and theta_m_1 = theta_m_2 of 6051-6058
      rotate_saves(ctx);
      swap_theta(ctx);
      relayout(false);
    }
    if (final_pending) {
      CHK(exchange_wait(ctx));
      final_pending = false;
    }
  }

  if (cf.scalar_advection && cf.split_dynamics_transport) {       // 1355-1576
    double rk_ts[3] = {dt / 3., dt / 2., dt};
    if (cf.time_integration_order == 2) rk_ts[0] = dt / 2.;
    const bool mono3 = cf.monotonic || cf.positive_definite;
    for (int rk_step = 1; rk_step <= 3; ++rk_step) {
      if (rk_step < 3 || !mono3) {
        EACH(advance_scalars(ctx, d, p, rk_ts[rk_step - 1], rk_step, true));
      } else {
        CHK(advance_scalars_mono(ctx, P, rk_ts[rk_step - 1], true, true));
      }
      if (lbc) CHK(lbc_scalars(ctx, P, dt, rk_ts[rk_step - 1]));  // 1491-1560
      if (rk_step == 2 && mono3) {
        // the rk3 limiter's preparation (3737-3777) reads scalars(tl1), scalars_tend, rho_zz(tl1),
        // ruAvg and wwAvg, none of which this exchange touches, and writes none of the scalars(tl2)
        // it moves: so it runs first and its scalars_old exchange (3757) rides with 1569-1572
        mono_prep(ctx, P, rk_ts[2], true);
        CHK(exchange(ctx, {{"state", "scalars", 2, ALL_LAYERS}, {"state", "scalars", 1, ALL_LAYERS}}));
      } else if (rk_step < 3) {
        CHK(exchange(ctx, {{"state", "scalars", 2, ALL_LAYERS}}));  // 1569-1572
      }
    }
  }
  EACH(reconstruct(ctx, d, p, p.u2));                              // mpas_reconstruct (1581-1603)
  if (ctx->physics & MPAS_DYC_PHYSICS_TENDENCIES) {                // DO_PHYSICS block, 1610-1648
    // rqvdynten (1629-1643) for cu_grell_freitas / cu_tiedtke / cu_ntiedtke, from the scalars before
    // the clip; the microphysics call itself (1650-1660) belongs to the host, after this step
    if (ctx->physics & MPAS_DYC_PHYSICS_RQVDYNTEN)
      EACH(LAUNCH(k_physics_rqvdynten, d.nCells + 1, d, p, ctx->index_qv, cf.monotonic, dt));
    for (auto& b : ctx->blk) {
      const int64_t n = (int64_t)b.d.ns * (b.d.nCells + 1) * b.d.K;
      if (!ctx->planning)
        hipLaunchKernelGGL(k_physics_clip_scalars, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)),
                           dim3(256), 0, ctx->stream, ::P<double>(ctx, b, "state", "scalars", 2), n);
    }
  }
  // the rest of the step follows the microphysics (1650-1660): when the host runs it, the host
  // calls mpas_dyc_finish_step after it
  if (!(ctx->physics & MPAS_DYC_PHYSICS_MICROPHYSICS)) CHK(step_tail(ctx, P, dt));
  return MPAS_DYC_OK;
}

// model init, mpas_atm_core.F:143-186 (exchanges) and 387-404 (the two routines)
// coupled = false: a restart (config_do_restart without DA cycling, 387-397) skips
// atm_init_coupled_diagnostics; the coupled state and its perturbations come from the restart file
int init_diagnostics(mpas_dyc_ctx* ctx, double dt, bool coupled = true) {
  const std::vector<Ptrs> P = block_ptrs(ctx);
  CHK(exchange(ctx, {{"state", "u", 1, ALL_LAYERS}}));           // 145
  if (coupled) {
    EACH(LAUNCH(k_init_coupled_a, d.nCells, d, p, ctx->index_qv));
    EACH(LAUNCH(k_init_coupled_b, d.nEdges, d, p));
    EACH(LAUNCH(k_init_coupled_c, d.nCells, d, p));
  }
  EACH(solve_diagnostics(ctx, d, p, dt, 1, 0));
  EACH(reconstruct(ctx, d, p, p.u1));                              // mpas_atm_core.F:411-421
  CHK(exchange(ctx, {{"diag", "pv_edge", 0, ALL_LAYERS}, {"diag", "ru", 0, ALL_LAYERS},  // 180-186
                     {"diag", "rw", 0, ALL_LAYERS}}));
  return MPAS_DYC_OK;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
namespace {

int fill_dims(Dims& d, const mpas_dyc_dims* dims) {
#ifdef MPAS_WIDE
  // column = one workgroup of WIDE_THREADS lanes (levels 0..K of w)
  // (the 128-lane build: 64..127 levels; the 256-lane build: 128..255; the 512-lane build: 256..511)
  constexpr int lo = WIDE_THREADS == 128 ? MPAS_DYC_MAX_LEVELS_WAVE
                     : WIDE_THREADS == 256 ? MPAS_DYC_MAX_LEVELS_WIDE : MPAS_DYC_MAX_LEVELS_256;
  if (dims->nVertLevels <= lo || dims->nVertLevels >= WIDE_THREADS || dims->nVertLevels > MPAS_DYC_MAX_LEVELS)
    return MPAS_DYC_EINVAL;
  static_assert(WIDE_THREADS == 128 || WIDE_THREADS == 256 || WIDE_THREADS == 512,
                "wide builds: 128, 256 or 512 lanes per column");
#else
  // column = one wavefront (levels 0..K of w)
  if (dims->nVertLevels < 4 || dims->nVertLevels > MPAS_DYC_MAX_LEVELS_WAVE) return MPAS_DYC_EINVAL;
#endif
  if (dims->maxEdges < 3 || dims->maxEdges2 < dims->maxEdges || dims->num_scalars < 1) return MPAS_DYC_EINVAL;
  if (dims->nCells < 1 || dims->nEdges < 1 || dims->nVertices < 1) return MPAS_DYC_EINVAL;
  if (dims->nCellsSolve < 1 || dims->nCellsSolve > dims->nCells || dims->nEdgesSolve > dims->nEdges ||
      dims->nVerticesSolve > dims->nVertices)
    return MPAS_DYC_EINVAL;
  d.nCells = dims->nCells;
  d.nEdges = dims->nEdges;
  d.nVertices = dims->nVertices;
  d.K = dims->nVertLevels;
  d.maxEdges = dims->maxEdges;
  d.maxEdges2 = dims->maxEdges2;
  d.ns = dims->num_scalars;
  d.nCellsSolve = dims->nCellsSolve;
  d.nEdgesSolve = dims->nEdgesSolve;
  d.nVerticesSolve = dims->nVerticesSolve;
  d.moist_start = dims->moist_start - 1;
  d.moist_end = dims->moist_end - 1;
  return MPAS_DYC_OK;
}

void fill_config(Config& c, const mpas_dyc_config* cfg) {
  c.time_integration_order = cfg->config_time_integration_order;
  c.number_of_sub_steps = cfg->config_number_of_sub_steps;
  c.dynamics_split_steps = cfg->config_dynamics_split_steps;
  c.number_rayleigh_damp_u_levels = cfg->config_number_rayleigh_damp_u_levels;
  c.split_dynamics_transport = cfg->config_split_dynamics_transport;
  c.scalar_advection = cfg->config_scalar_advection;
  c.positive_definite = cfg->config_positive_definite;
  c.monotonic = cfg->config_monotonic;
  c.mix_full = cfg->config_mix_full;
  c.rayleigh_damp_u = cfg->config_rayleigh_damp_u;
  c.horiz_mixing_smag = cfg->config_horiz_mixing;
  c.h_mom_eddy_visc2 = cfg->config_h_mom_eddy_visc2;
  c.h_mom_eddy_visc4 = cfg->config_h_mom_eddy_visc4;
  c.v_mom_eddy_visc2 = cfg->config_v_mom_eddy_visc2;
  c.h_theta_eddy_visc2 = cfg->config_h_theta_eddy_visc2;
  c.h_theta_eddy_visc4 = cfg->config_h_theta_eddy_visc4;
  c.v_theta_eddy_visc2 = cfg->config_v_theta_eddy_visc2;
  c.len_disp = cfg->config_len_disp;
  c.visc4_2dsmag = cfg->config_visc4_2dsmag;
  c.del4u_div_factor = cfg->config_del4u_div_factor;
  c.coef_3rd_order = cfg->config_coef_3rd_order;
  c.smagorinsky_coef = cfg->config_smagorinsky_coef;
  c.epssm = cfg->config_epssm;
  c.smdiv = cfg->config_smdiv;
  c.apvm_upwinding = cfg->config_apvm_upwinding;
  c.mpas_cam_coef = cfg->config_mpas_cam_coef;
  c.rayleigh_damp_u_timescale_days = cfg->config_rayleigh_damp_u_timescale_days;
}

int64_t target_n(const Block& b, Target t) {
  switch (t) {
    case T_CELL: return b.d.nCells;
    case T_EDGE: return b.d.nEdges;
    case T_VERTEX: return b.d.nVertices;
    default: return 0;
  }
}

Block* get_block(mpas_dyc_ctx* ctx, int32_t block) {
  if (!ctx || block < 0 || block >= (int32_t)ctx->blk.size()) return nullptr;
  return &ctx->blk[block];
}

// edges with at least one owned cell (the acoustic edge loop's active set), from MPAS 1-based cellsOnEdge
void count_active_edges(Block& b, const int32_t* coe) {
  int64_t n = 0;
  for (int e = 0; e < b.d.nEdges; ++e) {
    const int c1 = coe[2 * e] - 1, c2 = coe[2 * e + 1] - 1;
    if ((c1 >= 0 && c1 < b.d.nCellsSolve) || (c2 >= 0 && c2 < b.d.nCellsSolve)) ++n;
  }
  b.nEdges_act = n;
}

// build the exchange plans of both time-level parities of a step outside graph capture
// Run every plan's RCCL group once, eagerly, before the step is captured into a hipGraph: RCCL
// sets up a peer connection the first time a send/recv to that peer is enqueued, and that
// setup is kept out of stream capture.  Plans are visited in key order, which is the same on
// every rank (same srk3 sequence, same keys), so the sends and receives of each rank pair
// match.  The received bytes land in the receive buffers only (no unpack): they are scratch
// until the real exchange overwrites them.
int warm_rccl(mpas_dyc_ctx* ctx) {
  if (!ctx->comm) return MPAS_DYC_OK;
  bool any = false;
  for (auto& kv : ctx->plans) {
    XPlan& pl = kv.second;
    if (pl.warmed) continue;
    pl.warmed = true;
    if (pl.p2p || (pl.rsend.empty() && pl.rrecv.empty())) continue;
    set_last_key(ctx, "warm_rccl " + kv.first);
    CHK(rccl_group(ctx, pl));
    // one group at a time: a group that never completes names its plan in last_key
    HIPCHK(hipStreamSynchronize(ctx->stream));
    any = true;
  }
  (void)any;
  return MPAS_DYC_OK;
}

// One eager step with the exchange profile's events (mpas_dyc_set_profile), read back at its end
int profiled_step(mpas_dyc_ctx* ctx, double dt) {
  auto clear = [&]() {
    for (auto* v : {&ctx->prof_exposed, &ctx->prof_rccl}) {
      for (hipEvent_t e : *v) (void)hipEventDestroy(e);
      v->clear();
    }
  };
  clear();
  for (auto& e : ctx->prof_step)
    if (!e) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventRecord(ctx->prof_step[0], ctx->stream));
  ctx->graph_ran = false;
  const int r = srk3(ctx, dt);
  HIPCHK(hipEventRecord(ctx->prof_step[1], ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->xstream));
  auto sum = [&](const std::vector<hipEvent_t>& v) {
    double ms = 0.0;
    for (size_t i = 0; i + 1 < v.size(); i += 2) {
      float t = 0.f;
      if (hipEventElapsedTime(&t, v[i], v[i + 1]) == hipSuccess) ms += t;
    }
    return ms;
  };
  float tot = 0.f;
  (void)hipEventElapsedTime(&tot, ctx->prof_step[0], ctx->prof_step[1]);
  ctx->prof_out[0] = (double)(ctx->prof_exposed.size() / 2);
  ctx->prof_out[1] = tot;
  ctx->prof_out[2] = sum(ctx->prof_exposed);
  ctx->prof_out[3] = (double)(ctx->prof_rccl.size() / 2);
  ctx->prof_out[4] = sum(ctx->prof_rccl);
  clear();
  return r;
}

int plan_all(mpas_dyc_ctx* ctx, double dt) {
  if (!ctx->bnd_ready) CHK(compute_bnd(ctx));
  const std::string sig = layout_sig(ctx);
  if (!needs_exchange(ctx) || ctx->planned.count(sig)) return MPAS_DYC_OK;
  const Layout l = save_layout(ctx);  // the dry run rotates buffers as the step does
  ctx->planning = true;
  int r = srk3(ctx, dt);
  ctx->planning = false;
  restore_layout(l);
  if (r == MPAS_DYC_OK) {
    ctx->planned.insert(sig);
    r = ctx->p2p ? p2p_setup(ctx) : MPAS_DYC_OK;
    if (r == P2P_UNAVAILABLE) {  // every rank is here: plan again for RCCL
      if (!ctx->comm) return MPAS_DYC_ECOMM;  // mpas_dyc_comm_init_host: nothing to fall back to
      p2p_fallback(ctx);
      return plan_all(ctx, dt);
    }
    if (r == MPAS_DYC_OK) r = warm_rccl(ctx);
  }
  return r;
}

}  // namespace

extern "C" {

int mpas_dyc_create_blocks(int32_t nblocks, const mpas_dyc_dims* dims, const mpas_dyc_config* cfg, int device,
                           mpas_dyc_ctx** out) {
  if (!dims || !cfg || !out || nblocks < 1) return MPAS_DYC_EINVAL;
  *out = nullptr;
  mpas_dyc_ctx* ctx = new mpas_dyc_ctx();
  ctx->blk.resize(nblocks);
  for (int b = 0; b < nblocks; ++b) {
    if (fill_dims(ctx->blk[b].d, &dims[b]) != MPAS_DYC_OK || dims[b].nVertLevels != dims[0].nVertLevels ||
        dims[b].num_scalars != dims[0].num_scalars) {
      delete ctx;
      return MPAS_DYC_EINVAL;
    }
    ctx->blk[b].me_decl = dims[b].maxEdges;
    ctx->blk[b].me2_decl = dims[b].maxEdges2;
  }
  ctx->index_qv = dims[0].index_qv - 1;
  fill_config(ctx->cf, cfg);
  if (ctx->cf.time_integration_order != 2 && ctx->cf.time_integration_order != 3) {
    delete ctx;
    return MPAS_DYC_EINVAL;
  }
  if (device == MPAS_DYC_HOST_ONLY) {  // planner only: registry and dims, nothing on a device
    ctx->host_only = true;
    for (auto& b : ctx->blk) build_registry(b);
    *out = ctx;
    return MPAS_DYC_OK;
  }
  if (device >= 0 && hipSetDevice(device) != hipSuccess) {
    delete ctx;
    return MPAS_DYC_EHIP;
  }
  (void)hipGetDevice(&ctx->device);
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return MPAS_DYC_EHIP;
  }
  for (auto& e : ctx->ev) (void)hipEventCreate(&e);
  if (hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->xfork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->xjoin, hipEventDisableTiming) != hipSuccess) {
    mpas_dyc_destroy(ctx);
    return MPAS_DYC_EHIP;
  }
  if (const char* kt = getenv("MPAS_DYCORE_KERNELS")) {
    const std::string t(kt);
    g_kernel_tier = t == "general" ? 0 : t == "batched" ? 1 : 2;
  } else {
    g_kernel_tier = 2;
  }
  g_fuse_smlstep = 1;
  if (const char* fs = getenv("MPAS_DYCORE_FUSE_SMLSTEP")) g_fuse_smlstep = std::string(fs) != "0";
  g_mono_pairs = 1;
  if (const char* mp = getenv("MPAS_DYCORE_MONO_PAIRS")) g_mono_pairs = std::string(mp) != "0";
  g_delsq_pair = 1;
  if (const char* dp = getenv("MPAS_DYCORE_DELSQ_PAIR")) g_delsq_pair = std::string(dp) != "0";
  g_cells2_pair = 1;
  if (const char* cp = getenv("MPAS_DYCORE_CELLS2_PAIR")) g_cells2_pair = std::string(cp) != "0";
  g_cells1_pair = 1;
  if (const char* c1 = getenv("MPAS_DYCORE_CELLS1_PAIR")) g_cells1_pair = std::string(c1) != "0";
  g_mono_fuse = MONO_FUSE_BOUNDS;
  if (const char* mf = getenv("MPAS_DYCORE_MONO_FUSE")) g_mono_fuse = std::atoi(mf);
  if (const char* fp = getenv("MPAS_DYCORE_FUSED_PACK")) ctx->fused_pack_enabled = std::string(fp) != "0";
  if (const char* lb = getenv("MPAS_DYCORE_LOOPBACK")) ctx->loopback = std::atoi(lb);
  if (const char* pp = getenv("MPAS_DYCORE_P2P")) ctx->p2p = std::atoi(pp);
  if (const char* pm = getenv("MPAS_DYCORE_P2P_MERGE")) ctx->p2p_merge = std::atoi(pm) != 0;
  if (const char* pu = getenv("MPAS_DYCORE_P2P_PULL")) ctx->p2p_pull = std::atoi(pu) != 0;
  if (const char* li = getenv("MPAS_DYCORE_LATE_ISSUE")) ctx->late_issue = std::string(li) == "1";
  if (const char* oa = getenv("MPAS_DYCORE_OVERLAP_ALL")) ctx->overlap_all = std::string(oa) == "1";
  if (const char* ov = getenv("MPAS_DYCORE_OVERLAP")) ctx->overlap = std::atoi(ov);
  for (auto& b : ctx->blk) {
    build_registry(b);
    for (auto& f : b.fields) {
      if (f.lazy) continue;
      // 256 B of slack: the two-levels-per-lane kernels read 16 B at the last level of the last column
      const int64_t nb = field_bytes(b, f) + 256;
      for (int t = 0; t < f.ntl; ++t) {
        if (hipMalloc(&f.buf[t], nb) != hipSuccess || hipMemset(f.buf[t], 0, nb) != hipSuccess) {
          mpas_dyc_destroy(ctx);
          return MPAS_DYC_EHIP;
        }
      }
      if (is_host_0d(f)) f.buf[1] = new double(0.0);  // host mirror of the 0-d field
    }
    const size_t nf = 2 + (size_t)b.d.ns;
    if (hipMalloc(&b.sum_part, (size_t)SUM_MAX_FIELDS * SUM_PARTS * SUM_REC * sizeof(double)) != hipSuccess ||
        hipMalloc(&b.sum_out, nf * SUM_REC * sizeof(double)) != hipSuccess) {
      mpas_dyc_destroy(ctx);
      return MPAS_DYC_EHIP;
    }
  }
  *out = ctx;
  return MPAS_DYC_OK;
}

int mpas_dyc_create(const mpas_dyc_dims* dims, const mpas_dyc_config* cfg, int device, mpas_dyc_ctx** out) {
  return mpas_dyc_create_blocks(1, dims, cfg, device, out);
}

void mpas_dyc_destroy(mpas_dyc_ctx* ctx) {
  if (!ctx) return;
  if (ctx->host_only) {
    delete ctx;
    return;
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (getenv("MPAS_DYCORE_P2P_DEBUG"))  // every one-sided exchange point's use count (ranks compare them)
    for (const auto& kv : ctx->plans)
      if (kv.second.p2p_id >= 0 && kv.second.p2p_cnt) {
        unsigned long long c[2] = {0, 0};
        (void)hipMemcpy(c, kv.second.p2p_cnt, sizeof(c), hipMemcpyDeviceToHost);
        printf("p2pdbg rank %d id %d uses %llu wg %llu nget %d %s\n", ctx->rank, kv.second.p2p_id, c[0], c[1],
               kv.second.nget, kv.first.c_str());
      }
  invalidate_plans(ctx);
  for (auto& b : ctx->blk) {
    for (auto& f : b.fields) {
      for (int t = 0; t < f.ntl; ++t)
        if (f.buf[t]) (void)hipFree(f.buf[t]);
      if (f.packed) (void)hipFree(f.packed);
      if (is_host_0d(f)) delete (double*)f.buf[1];
    }
    for (auto& x : b.xl) {
      if (x.d_idx) (void)hipFree(x.d_idx);
      if (x.d_pos) (void)hipFree(x.d_pos);
    }
    if (b.sum_part) (void)hipFree(b.sum_part);
    if (b.sum_out) (void)hipFree(b.sum_out);
  }
  if (ctx->sum_gather) (void)hipFree(ctx->sum_gather);
  for (void* p : ctx->p2p_mapped) (void)hipIpcCloseMemHandle(p);
  if (ctx->p2p_flags) (void)hipFree(ctx->p2p_flags);
  if (ctx->p2p_status) (void)hipFree(ctx->p2p_status);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->prof_step)
    if (e) (void)hipEventDestroy(e);
  if (ctx->xfork) (void)hipEventDestroy(ctx->xfork);
  if (ctx->xjoin) (void)hipEventDestroy(ctx->xjoin);
  if (ctx->xstream) (void)hipStreamDestroy(ctx->xstream);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* mpas_dyc_last_error(const mpas_dyc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int32_t mpas_dyc_num_blocks(const mpas_dyc_ctx* ctx) { return ctx ? (int32_t)ctx->blk.size() : 0; }

int64_t mpas_dyc_block_field_bytes(const mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name) {
  if (!ctx || !pool || !name || block < 0 || block >= (int32_t)ctx->blk.size()) return 0;
  const Block& b = ctx->blk[block];
  auto it = b.by_name.find(std::string(pool) + "." + name);
  if (it == b.by_name.end()) return 0;
  return field_bytes(b, b.fields[it->second]);
}

int64_t mpas_dyc_field_bytes(const mpas_dyc_ctx* ctx, const char* pool, const char* name) {
  return mpas_dyc_block_field_bytes(ctx, 0, pool, name);
}

void* mpas_dyc_block_field_device_ptr(mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name,
                                      int32_t time_level) {
  Block* b = get_block(ctx, block);
  if (!b || !pool || !name) return nullptr;
  Field* f = find(*b, pool, name);
  if (!f) return nullptr;
  // the kernels read packed copies of the maxEdges-strided mesh fields (pack_mesh) and zb_cell / zb3_cell
  // through zb_p / zb_m: a caller may write through the pointer, so the next step packs them again
  if (f->me || (f->pool == "mesh" && (f->name == "zb_cell" || f->name == "zb3_cell"))) ctx->bnd_ready = false;
  return f->buf[slot_of(ctx, *f, time_level)];
}

void* mpas_dyc_field_device_ptr(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level) {
  return mpas_dyc_block_field_device_ptr(ctx, 0, pool, name, time_level);
}

int mpas_dyc_set_block_field(mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name,
                             int32_t time_level, const void* host, int64_t nbytes) {
  if (!ctx || !pool || !name || !host) return MPAS_DYC_EINVAL;
  if (ctx->host_only) {
    ctx->err = "host-only context holds no fields";
    return MPAS_DYC_ESTATE;
  }
  Block* bp = get_block(ctx, block);
  if (!bp) {
    ctx->err = "no block " + std::to_string(block);
    return MPAS_DYC_EINVAL;
  }
  Block& b = *bp;
  Field* f = find(b, pool, name);
  if (!f) {
    ctx->err = std::string("unknown field ") + pool + "." + name;
    return MPAS_DYC_EINVAL;
  }
  if (is_host_0d(*f)) {
    if (nbytes != 8) return MPAS_DYC_EINVAL;
    *(double*)f->buf[1] = *(const double*)host;
    HIPCHK(hipMemcpy(f->buf[0], host, 8, hipMemcpyHostToDevice));
    return MPAS_DYC_OK;
  }
  const int64_t nb = field_bytes(b, *f);
  if (nbytes != nb) {
    ctx->err = "size mismatch for " + f->pool + "." + f->name + ": got " + std::to_string(nbytes) + " expected " +
               std::to_string(nb);
    return MPAS_DYC_EINVAL;
  }
  const int slot = slot_of(ctx, *f, time_level);
  HIPCHK(hipSetDevice(ctx->device));
  if (f->lazy && !f->buf[slot]) HIPCHK(hipMalloc(&f->buf[slot], nb + 256));
  if (f->me) ctx->bnd_ready = false;  // pack_mesh copies the new image for the kernels
  if (f->is_int && f->target != T_NONE) {
    // MPAS 1-based -> device 0-based; out-of-range / 0 -> garbage slot
    const int64_t n = field_elems(b, *f);
    std::vector<int32_t> tmp(n);
    const int32_t* src = (const int32_t*)host;
    const int64_t nt = target_n(b, f->target);
    for (int64_t i = 0; i < n; ++i) {
      int32_t v = src[i] - 1;
      if (f->target == T_SMALL) v = v < 0 ? 0 : v;
      else if (v < 0 || v > nt) v = (int32_t)nt;
      tmp[i] = v;
    }
    if (f->pool == "mesh" && f->name == "cellsOnEdge") {
      count_active_edges(b, src);
      b.h_coe = tmp;
      ctx->bnd_ready = false;
    }
    if (f->pool == "mesh" && f->name == "edgesOnCell") {
      b.h_eoc = tmp;
      ctx->bnd_ready = false;
    }
    if (f->pool == "mesh" && (f->name == "verticesOnEdge" || f->name == "edgesOnVertex")) {
      (f->name == "verticesOnEdge" ? b.h_voe : b.h_eov) = tmp;
      if (!ctx->plans.empty()) invalidate_plans(ctx);  // the fused u exchange's write-back vertices
    }
    HIPCHK(hipMemcpyAsync(f->buf[slot], tmp.data(), nb, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  } else if (f->nsub > 1) {
    // Fortran (nsub, inner/nsub, n+1) -> scalar-major [nsub][n+1][inner/nsub]
    const int64_t n = nloc(b, f->loc), ns = f->nsub, m = f->inner / ns;
    const double* src = (const double*)host;
    std::vector<double> tmp(n * f->inner);
    for (int64_t c = 0; c < n; ++c)
      for (int64_t k = 0; k < m; ++k)
        for (int64_t s = 0; s < ns; ++s) tmp[(s * n + c) * m + k] = src[(c * m + k) * ns + s];
    HIPCHK(hipMemcpyAsync(f->buf[slot], tmp.data(), nb, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  } else {
    HIPCHK(hipMemcpyAsync(f->buf[slot], host, nb, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (f->pool == "mesh" && f->name == "nEdgesOnCell") {
      b.h_noc.assign((const int32_t*)host, (const int32_t*)host + nb / 4);
      ctx->bnd_ready = false;
    }
    if (f->pool == "mesh" && f->name == "nEdgesOnEdge") {
      b.h_noe.assign((const int32_t*)host, (const int32_t*)host + nb / 4);
      ctx->bnd_ready = false;
    }
    if (f->pool == "mesh" && (f->name == "zb_cell" || f->name == "zb3_cell")) ctx->bnd_ready = false;  // zb_p / zb_m
    if (f->pool == "tend" && f->name == "rt_diabatic_tend") {
      const double* h = (const double*)host;
      int nz = 0;
      for (int64_t i = 0; i < nb / 8 && !nz; ++i) nz = h[i] != 0.0;
      b.d.diabatic = nz;
    }
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_set_field(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level,
                       const void* host, int64_t nbytes) {
  return mpas_dyc_set_block_field(ctx, 0, pool, name, time_level, host, nbytes);
}

int mpas_dyc_get_block_field(mpas_dyc_ctx* ctx, int32_t block, const char* pool, const char* name,
                             int32_t time_level, void* host, int64_t nbytes) {
  if (!ctx || !pool || !name || !host) return MPAS_DYC_EINVAL;
  if (ctx->host_only) {
    ctx->err = "host-only context holds no fields";
    return MPAS_DYC_ESTATE;
  }
  Block* bp = get_block(ctx, block);
  if (!bp) {
    ctx->err = "no block " + std::to_string(block);
    return MPAS_DYC_EINVAL;
  }
  Block& b = *bp;
  Field* f = find(b, pool, name);
  if (!f) {
    ctx->err = std::string("unknown field ") + pool + "." + name;
    return MPAS_DYC_EINVAL;
  }
  if (is_host_0d(*f)) {
    if (nbytes != 8) return MPAS_DYC_EINVAL;
    *(double*)host = *(double*)f->buf[1];
    return MPAS_DYC_OK;
  }
  const int64_t nb = field_bytes(b, *f);
  if (nbytes != nb) {
    ctx->err = "size mismatch for " + f->pool + "." + f->name;
    return MPAS_DYC_EINVAL;
  }
  if (!f->buf[slot_of(ctx, *f, time_level)]) {
    ctx->err = f->pool + "." + f->name + " has not been set";
    return MPAS_DYC_ESTATE;
  }
  HIPCHK(hipSetDevice(ctx->device));
  if (f->nsub > 1) {  // scalar-major -> Fortran (nsub, inner/nsub, n+1)
    const int64_t n = nloc(b, f->loc), ns = f->nsub, m = f->inner / ns;
    std::vector<double> tmp(n * f->inner);
    HIPCHK(hipMemcpyAsync(tmp.data(), f->buf[slot_of(ctx, *f, time_level)], nb, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    double* dst = (double*)host;
    for (int64_t c = 0; c < n; ++c)
      for (int64_t k = 0; k < m; ++k)
        for (int64_t s = 0; s < ns; ++s) dst[(c * m + k) * ns + s] = tmp[(s * n + c) * m + k];
    return MPAS_DYC_OK;
  }
  HIPCHK(hipMemcpyAsync(host, f->buf[slot_of(ctx, *f, time_level)], nb, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (f->is_int && f->target != T_NONE) {
    int32_t* h = (int32_t*)host;
    const int64_t n = field_elems(b, *f);
    for (int64_t i = 0; i < n; ++i) h[i] += 1;
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_get_field(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level, void* host,
                       int64_t nbytes) {
  return mpas_dyc_get_block_field(ctx, 0, pool, name, time_level, host, nbytes);
}

int mpas_dyc_set_exchange_list(mpas_dyc_ctx* ctx, int32_t block, int32_t location, int32_t halo_layer,
                               int32_t direction, int32_t peer_rank, int32_t peer_block, const int32_t* local_index,
                               int32_t n) {
  Block* bp = get_block(ctx, block);
  if (!bp) {
    if (ctx) ctx->err = "no block " + std::to_string(block);
    return MPAS_DYC_EINVAL;
  }
  if (location < MPAS_DYC_CELL || location > MPAS_DYC_VERTEX || halo_layer < 1 || halo_layer > 3 ||
      (location == MPAS_DYC_CELL && halo_layer > 2) || (direction != MPAS_DYC_SEND && direction != MPAS_DYC_RECV) ||
      peer_rank < 0 || peer_block < 0 || n < 0 || (n > 0 && !local_index)) {
    ctx->err = "invalid exchange list arguments";
    return MPAS_DYC_EINVAL;
  }
  Block& b = *bp;
  const int64_t nl = location == MPAS_DYC_CELL ? b.d.nCells : location == MPAS_DYC_EDGE ? b.d.nEdges : b.d.nVertices;
  const int64_t nown = location == MPAS_DYC_CELL ? b.d.nCellsSolve
                       : location == MPAS_DYC_EDGE ? b.d.nEdgesSolve : b.d.nVerticesSolve;
  std::vector<int32_t> idx(n);
  for (int i = 0; i < n; ++i) {
    const int32_t v = local_index[i] - 1;
    // senders send owned elements; receivers fill halo elements
    const bool ok = direction == MPAS_DYC_SEND ? (v >= 0 && v < nown) : (v >= nown && v < nl);
    if (!ok) {
      ctx->err = "exchange list index " + std::to_string(local_index[i]) + " out of range";
      return MPAS_DYC_EINVAL;
    }
    idx[i] = v;
  }
  invalidate_plans(ctx);
  XList* x = nullptr;
  for (auto& e : b.xl)
    if (e.loc == location && e.layer == halo_layer && e.dir == direction && e.peer_rank == peer_rank &&
        e.peer_block == peer_block)
      x = &e;
  if (!x) {
    b.xl.push_back(XList{location, halo_layer, direction, peer_rank, peer_block});
    x = &b.xl.back();
  }
  if (x->d_idx && !ctx->host_only) {
    HIPCHK(hipFree(x->d_idx));
    x->d_idx = nullptr;
  }
  x->n = n;
  x->h_idx = idx;
  if (n > 0 && !ctx->host_only) {
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMalloc(&x->d_idx, n * sizeof(int32_t)));
    HIPCHK(hipMemcpy(x->d_idx, idx.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_set_exchange_positions(mpas_dyc_ctx* ctx, int32_t block, int32_t location, int32_t halo_layer,
                                    int32_t direction, int32_t peer_rank, const int32_t* local_index,
                                    const int32_t* position, int32_t n) {
  Block* bp = get_block(ctx, block);
  if (!bp) {
    if (ctx) ctx->err = "no block " + std::to_string(block);
    return MPAS_DYC_EINVAL;
  }
  if (location < MPAS_DYC_CELL || location > MPAS_DYC_VERTEX || halo_layer < 1 || halo_layer > 3 ||
      (location == MPAS_DYC_CELL && halo_layer > 2) || (direction != MPAS_DYC_SEND && direction != MPAS_DYC_RECV) ||
      peer_rank < 0 || n < 0 || (n > 0 && (!local_index || !position))) {
    ctx->err = "invalid exchange list arguments";
    return MPAS_DYC_EINVAL;
  }
  if (peer_rank == ctx->rank && !ctx->host_only && ctx->nranks > 1) {
    ctx->err = "positional lists are for other ranks (mpas_dyc_set_exchange_list copies within a process)";
    return MPAS_DYC_EINVAL;
  }
  Block& b = *bp;
  const int64_t nl = location == MPAS_DYC_CELL ? b.d.nCells : location == MPAS_DYC_EDGE ? b.d.nEdges : b.d.nVertices;
  const int64_t nown = location == MPAS_DYC_CELL ? b.d.nCellsSolve
                       : location == MPAS_DYC_EDGE ? b.d.nEdgesSolve : b.d.nVerticesSolve;
  std::vector<int32_t> idx(n), pos(n);
  std::set<int32_t> seen;
  for (int i = 0; i < n; ++i) {
    const int32_t v = local_index[i] - 1;
    const bool ok = direction == MPAS_DYC_SEND ? (v >= 0 && v < nown) : (v >= nown && v < nl);
    if (!ok || position[i] < 1 || !seen.insert(position[i]).second) {
      ctx->err = "exchange list entry " + std::to_string(i + 1) + " (index " + std::to_string(local_index[i]) +
                 ", position " + std::to_string(position[i]) + ") out of range or repeated";
      return MPAS_DYC_EINVAL;
    }
    idx[i] = v;
    pos[i] = position[i] - 1;
  }
  invalidate_plans(ctx);
  XList* x = nullptr;
  for (auto& e : b.xl)
    if (e.loc == location && e.layer == halo_layer && e.dir == direction && e.peer_rank == peer_rank &&
        e.peer_block < 0)
      x = &e;
  if (!x) {
    b.xl.push_back(XList{location, halo_layer, direction, peer_rank, -1});
    x = &b.xl.back();
  }
  if (!ctx->host_only) {
    if (x->d_idx) HIPCHK(hipFree(x->d_idx));
    if (x->d_pos) HIPCHK(hipFree(x->d_pos));
    x->d_idx = x->d_pos = nullptr;
  }
  x->n = n;
  x->h_idx = idx;
  x->h_pos = pos;
  if (n > 0 && !ctx->host_only) {
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMalloc(&x->d_idx, n * sizeof(int32_t)));
    HIPCHK(hipMemcpy(x->d_idx, idx.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&x->d_pos, n * sizeof(int32_t)));
    HIPCHK(hipMemcpy(x->d_pos, pos.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_comm_unique_id(void* id, int64_t nbytes) {
  if (!id || nbytes < (int64_t)sizeof(ncclUniqueId)) return MPAS_DYC_EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return MPAS_DYC_ECOMM;
  memcpy(id, &u, sizeof(u));
  return MPAS_DYC_OK;
}

int64_t mpas_dyc_comm_unique_id_bytes(void) { return (int64_t)sizeof(ncclUniqueId); }

int mpas_dyc_comm_init(mpas_dyc_ctx* ctx, const void* id, int64_t nbytes, int32_t nranks, int32_t rank) {
  if (!ctx || !id || nbytes < (int64_t)sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
    return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  invalidate_plans(ctx);
  if (ctx->comm) {
    ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  NCCLCHK(ncclCommInitRank(&ctx->comm, nranks, u, rank));
  ctx->nranks = nranks;
  ctx->rank = rank;
  return MPAS_DYC_OK;
}

int mpas_dyc_comm_init_host(mpas_dyc_ctx* ctx, int32_t nranks, int32_t rank, mpas_dyc_allgather_fn fn, void* user) {
  if (!ctx || !fn || nranks < 1 || rank < 0 || rank >= nranks) return MPAS_DYC_EINVAL;
  if (ctx->host_only || ctx->comm) return MPAS_DYC_ESTATE;
  invalidate_plans(ctx);
  ctx->host_allgather = fn;
  ctx->host_user = user;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->p2p = 1;
  return MPAS_DYC_OK;
}

int mpas_dyc_set_transport(mpas_dyc_ctx* ctx, int32_t rccl_for_local_blocks) {
  if (!ctx) return MPAS_DYC_EINVAL;
  invalidate_plans(ctx);
  ctx->rccl_local = rccl_for_local_blocks != 0;
  return MPAS_DYC_OK;
}

int mpas_dyc_halo_exchange(mpas_dyc_ctx* ctx, const char* pool, const char* name, int32_t time_level,
                           int32_t layer_mask) {
  if (!ctx || !pool || !name || layer_mask <= 0 || layer_mask > 7) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  std::string sp(pool), sn(name);
  // a plain exchange: its own plan (key suffix), never one whose pack / unpack a kernel of the step does
  ctx->plain_exchange = true;
  int r = exchange(ctx, {{sp.c_str(), sn.c_str(), time_level, (unsigned)layer_mask}});
  ctx->plain_exchange = false;
  if (r) return r;
  HIPCHK(hipGetLastError());
  for (auto& b : ctx->blk) {
    const Field* f = find(b, pool, name);
    if (f && f->me) ctx->bnd_ready = false;  // a maxEdges-strided mesh field: pack_mesh copies it again
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_set_summary(mpas_dyc_ctx* ctx, int32_t flags) {
  const int all = MPAS_DYC_PRINT_GLOBAL_MINMAX_VEL | MPAS_DYC_PRINT_DETAILED_MINMAX_VEL | MPAS_DYC_PRINT_GLOBAL_MINMAX_SCA;
  if (!ctx || (flags & ~all)) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->summary_flags = flags;
  ctx->summary_tl = 0;
  drop_graphs(ctx);  // captured steps bake the modes in
  return MPAS_DYC_OK;
}

namespace {
// blocks < 0: every block of the process folded; else that block alone (each reduced over ranks)
static int get_summary(mpas_dyc_ctx* ctx, int32_t blocks, mpas_dyc_summary* out, double* scalar_minmax, int32_t n) {
  if (!ctx || !out || blocks >= (int32_t)ctx->blk.size()) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  const int ns = ctx->blk[0].d.ns;
  if (scalar_minmax && n < 2 * ns) return MPAS_DYC_EINVAL;
  if (ctx->tail_pending) {  // the records would describe the step before, if any
    ctx->err = "no summary: with MPAS_DYC_PHYSICS_MICROPHYSICS, call mpas_dyc_finish_step after the step first";
    return MPAS_DYC_ESTATE;
  }
  if (!ctx->summary_flags || !ctx->summary_tl) {
    ctx->err = "no summary: no step has run with summary modes on (mpas_dyc_set_summary)";
    return MPAS_DYC_ESTATE;
  }
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  // Per field a payload of three located extremes (min, max, wind-speed max), each
  // (value, index, k, lat, lon) as the reference's localVals, then min0, max0, NaN count.
  const int nf = 2 + ns, PL = 18;
  std::vector<double> pay((size_t)nf * PL);
  auto fold = [&](double* acc, const double* x) {
    for (int e = 0; e < 3; ++e) {  // MPI_MINLOC / MPI_MAXLOC per attribute (mpas_dmpar.F:1106, 1154)
      double* a = acc + 5 * e;
      const double* b = x + 5 * e;
      const bool is_min = e == 0;
      if (is_min ? b[0] < a[0] : b[0] > a[0]) {
        for (int i = 0; i < 5; ++i) a[i] = b[i];
      } else if (b[0] == a[0]) {
        for (int i = 1; i < 5; ++i) a[i] = std::min(a[i], b[i]);
      }
    }
    acc[15] = std::min(acc[15], x[15]);
    acc[16] = std::max(acc[16], x[16]);
    acc[17] += x[17];
  };
  for (size_t ib = blocks < 0 ? 0 : (size_t)blocks; ib < (blocks < 0 ? ctx->blk.size() : (size_t)blocks + 1); ++ib) {
    Block& b = ctx->blk[ib];
    const bool first_block = ib == (blocks < 0 ? 0 : (size_t)blocks);
    std::vector<double> rec((size_t)nf * SUM_REC);
    HIPCHK(hipMemcpy(rec.data(), b.sum_out, rec.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int f = 0; f < nf; ++f) {
      const double* r = &rec[(size_t)f * SUM_REC];
      double x[PL];
      auto ext = [&](double* o, double v, double idx, double lat, double lon) {
        const long long i = (long long)idx;
        o[0] = v;
        o[1] = i >= 0 ? (double)(i / b.d.K + 1) : -1.0;  // indexMax
        o[2] = i >= 0 ? (double)(i % b.d.K + 1) : -1.0;  // kMax
        o[3] = lat;
        o[4] = lon;
      };
      ext(x, r[SR_MIN], r[SR_IMIN], r[SR_LAT_MIN], r[SR_LON_MIN]);
      ext(x + 5, r[SR_MAX], r[SR_IMAX], r[SR_LAT_MAX], r[SR_LON_MAX]);
      ext(x + 10, r[SR_SPD], r[SR_ISPD], r[SR_LAT_SPD], r[SR_LON_SPD]);
      x[15] = r[SR_MIN0];
      x[16] = r[SR_MAX0];
      x[17] = r[SR_NAN];
      double* acc = &pay[(size_t)f * PL];
      if (first_block) std::copy(x, x + PL, acc);
      else fold(acc, x);
    }
  }
  if (!ctx->comm && ctx->host_allgather && ctx->nranks > 1) {  // the host's all-gather, folded in rank order
    std::vector<char> all;
    CHK(allgather_bytes(ctx, pay.data(), pay.size() * sizeof(double), all));
    const size_t cnt = pay.size();
    const double* a = (const double*)all.data();
    std::copy(a, a + cnt, pay.begin());
    for (int r = 1; r < ctx->nranks; ++r)
      for (int f = 0; f < nf; ++f) fold(&pay[(size_t)f * PL], &a[cnt * r + (size_t)f * PL]);
  }
  if (ctx->comm && ctx->nranks > 1) {
    // all ranks' payloads to every rank (RCCL all-gather, in place), folded in rank order
    const size_t cnt = pay.size();
    if (!ctx->sum_gather) HIPCHK(hipMalloc(&ctx->sum_gather, cnt * ctx->nranks * sizeof(double)));
    HIPCHK(hipMemcpy(ctx->sum_gather + cnt * ctx->rank, pay.data(), cnt * sizeof(double), hipMemcpyHostToDevice));
    NCCLCHK(ncclAllGather(ctx->sum_gather + cnt * ctx->rank, ctx->sum_gather, cnt, ncclFloat64, ctx->comm, ctx->stream));
    std::vector<double> all(cnt * ctx->nranks);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(all.data(), ctx->sum_gather, all.size() * sizeof(double), hipMemcpyDeviceToHost));
    std::copy(all.begin(), all.begin() + cnt, pay.begin());
    for (int r = 1; r < ctx->nranks; ++r)
      for (int f = 0; f < nf; ++f) fold(&pay[(size_t)f * PL], &all[cnt * r + (size_t)f * PL]);
  }
  const double pi_const = 2.0 * asin(1.0);
  auto located = [&](const double* x) {
    mpas_dyc_extreme e;
    e.value = x[0];
    e.index = (int32_t)x[1];
    e.k = (int32_t)x[2];
    e.lat = x[3] * 180.0 / pi_const;  // 6769-6773
    e.lon = x[4] * 180.0 / pi_const;
    if (e.lon > 180.0) e.lon = e.lon - 360.0;
    return e;
  };
  *out = mpas_dyc_summary{};
  out->flags = ctx->summary_flags;
  const double* w = &pay[0];
  const double* u = &pay[PL];
  out->w_min = w[15];
  out->w_max = w[16];
  out->u_min = u[15];
  out->u_max = u[16];
  out->w_min_at = located(w);
  out->w_max_at = located(w + 5);
  out->u_min_at = located(u);
  out->u_max_at = located(u + 5);
  out->wsp_max_at = located(u + 10);
  out->nan_w = (int64_t)w[17];
  out->nan_u = (int64_t)u[17];
  if (scalar_minmax)
    for (int is = 0; is < ns; ++is) {
      scalar_minmax[2 * is] = pay[(size_t)(2 + is) * PL + 15];
      scalar_minmax[2 * is + 1] = pay[(size_t)(2 + is) * PL + 16];
    }
  return MPAS_DYC_OK;
}
}  // namespace

int mpas_dyc_get_summary(mpas_dyc_ctx* ctx, mpas_dyc_summary* out, double* scalar_minmax, int32_t n) {
  return get_summary(ctx, -1, out, scalar_minmax, n);
}

int mpas_dyc_get_block_summary(mpas_dyc_ctx* ctx, int32_t block, mpas_dyc_summary* out, double* scalar_minmax,
                               int32_t n) {
  if (block < 0) return MPAS_DYC_EINVAL;
  return get_summary(ctx, block, out, scalar_minmax, n);
}

int mpas_dyc_init_diagnostics(mpas_dyc_ctx* ctx, double dt) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->bnd_ready) CHK(compute_bnd(ctx));
  int r = init_diagnostics(ctx, dt);
  HIPCHK(hipGetLastError());
  return r;
}

int mpas_dyc_solve_diagnostics(mpas_dyc_ctx* ctx, double dt) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->bnd_ready) CHK(compute_bnd(ctx));
  int r = init_diagnostics(ctx, dt, false);
  HIPCHK(hipGetLastError());
  return r;
}

int mpas_dyc_set_lbc(mpas_dyc_ctx* ctx, int32_t apply, double seconds_to_interval_end) {
  if (!ctx || (apply != 0 && apply != 1)) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  // the mesh decides the kernel layout (pack_mesh); before it is known, compute_bnd checks
  if (apply && ctx->bnd_ready) {
    for (auto& b : ctx->blk)
      if (!pair_layout(b.d)) {
        ctx->err = lbc_layout_error(b.d);
        return MPAS_DYC_EINVAL;
      }
  }
  if ((apply != 0) != ctx->lbc) {  // other exchange points and kernels: re-plan, re-capture
    ctx->lbc = apply != 0;
    for (auto& b : ctx->blk) b.d.lbc = apply;
    invalidate_plans(ctx);
  }
  // the interval-end distance, ordered with the steps on the compute stream (a captured step reads it)
  for (auto& b : ctx->blk)
    hipLaunchKernelGGL(k_set_f64, dim3(1), dim3(1), 0, ctx->stream, P<double>(ctx, b, "lbc", "dtr"),
                       seconds_to_interval_end);
  HIPCHK(hipGetLastError());
  return MPAS_DYC_OK;
}

int mpas_dyc_set_physics(mpas_dyc_ctx* ctx, int32_t flags) {
  if (!ctx || (flags & ~(MPAS_DYC_PHYSICS_TENDENCIES | MPAS_DYC_PHYSICS_RQVDYNTEN | MPAS_DYC_PHYSICS_MICROPHYSICS)))
    return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  if ((flags & MPAS_DYC_PHYSICS_RQVDYNTEN) && !(flags & MPAS_DYC_PHYSICS_TENDENCIES)) return MPAS_DYC_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->physics = flags;
  for (auto& b : ctx->blk) b.d.physics = (flags & MPAS_DYC_PHYSICS_TENDENCIES) ? 1 : 0;
  drop_graphs(ctx);  // captured steps bake the flags in
  return MPAS_DYC_OK;
}

int mpas_dyc_model_init(mpas_dyc_ctx* ctx, int32_t h_scale_with_mesh, double config_zd, double config_xnutr) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  for (auto& b : ctx->blk) {
    for (const char* n : {"deriv_two", "zb", "zb3", "meshDensity", "areaCell", "areaTriangle"})
      if (!find(b, "mesh", n)->buf[0]) {
        ctx->err = std::string("mpas_dyc_model_init needs mesh.") + n + " (set it first)";
        return MPAS_DYC_ESTATE;
      }
    // the declared-stride images (buf), not the kernels' packed copies: pack_mesh redoes those after
    auto I = [&](const char* n) { return (int*)find(b, "mesh", n)->buf[0]; };
    auto R = [&](const char* n) { return (double*)find(b, "mesh", n)->buf[0]; };
    // k_mi_adv_compression keeps a cell's stencil list (at most 2 + 2 (maxEdges - 1) cells) in 20 slots and
    // reads deriv_two's 15 weights per side: cells of more than 10 edges are refused here
    int maxdeg = 0;
    for (int c = 0; c < b.d.nCells && c < (int)b.h_noc.size(); ++c) maxdeg = std::max(maxdeg, b.h_noc[c]);
    if ((int)b.h_noc.size() < b.d.nCells || maxdeg > 10) {
      ctx->err = "mpas_dyc_model_init: nEdgesOnCell " +
                 ((int)b.h_noc.size() < b.d.nCells ? std::string("not set") : "max " + std::to_string(maxdeg) + " > 10");
      return MPAS_DYC_EINVAL;
    }
    MInit m{};
    m.root4_cell = R("meshDensity_root4");
    m.root4_edge = R("meshDensityEdge_root4");
    m.dss_sin = R("dss_sin");
    m.nEdgesOnCell = I("nEdgesOnCell");
    m.edgesOnCell = I("edgesOnCell");
    m.cellsOnCell = I("cellsOnCell");
    m.verticesOnCell = I("verticesOnCell");
    m.cellsOnEdge = I("cellsOnEdge");
    m.verticesOnEdge = I("verticesOnEdge");
    m.cellsOnVertex = I("cellsOnVertex");
    m.edgesOnVertex = I("edgesOnVertex");
    m.deriv_two = R("deriv_two");
    m.zb = R("zb");
    m.zb3 = R("zb3");
    m.meshDensity = R("meshDensity");
    m.areaCell = R("areaCell");
    m.areaTriangle = R("areaTriangle");
    m.dcEdge = R("dcEdge");
    m.dvEdge = R("dvEdge");
    m.zgrid = R("zgrid");
    m.invAreaCell = R("invAreaCell");
    m.invDvEdge = R("invDvEdge");
    m.invDcEdge = R("invDcEdge");
    m.invAreaTriangle = R("invAreaTriangle");
    m.edgesOnVertex_sign = R("edgesOnVertex_sign");
    m.edgesOnCell_sign = R("edgesOnCell_sign");
    m.zb_cell = R("zb_cell");
    m.zb3_cell = R("zb3_cell");
    m.kiteForCell = I("kiteForCell");
    m.nAdvCellsForEdge = I("nAdvCellsForEdge");
    m.advCellsForEdge = I("advCellsForEdge");
    m.adv_coefs = R("adv_coefs");
    m.adv_coefs_3rd = R("adv_coefs_3rd");
    m.meshScalingDel2 = R("meshScalingDel2");
    m.meshScalingDel4 = R("meshScalingDel4");
    m.meshScalingRegionalCell = R("meshScalingRegionalCell");
    m.meshScalingRegionalEdge = R("meshScalingRegionalEdge");
    m.dss = R("dss");
    m.nCells = b.d.nCells;
    m.nEdges = b.d.nEdges;
    m.nVertices = b.d.nVertices;
    m.K = b.d.K;
    m.maxEdges = b.me_decl;
    auto grid = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    const int nmax = std::max(b.d.nCells, std::max(b.d.nEdges, b.d.nVertices));
    hipStream_t st = ctx->stream;
    // atm_mpas_init_block's order (mpas_atm_core.F:311-458): signs, inverses, adv_coef compression,
    // 3rd-order coupling, mesh scaling, damping coefficients
    hipLaunchKernelGGL(k_mi_vertex_signs, grid(b.d.nVertices), dim3(256), 0, st, m);
    hipLaunchKernelGGL(k_mi_cell_signs, grid((int64_t)b.d.nCells * b.me_decl), dim3(256), 0, st, m);
    hipLaunchKernelGGL(k_mi_inverses, grid(nmax), dim3(256), 0, st, m);
    hipLaunchKernelGGL(k_mi_adv_compression, grid(b.d.nEdges), dim3(256), 0, st, m);
    const double c3 = ctx->cf.coef_3rd_order;
    hipLaunchKernelGGL(k_mi_couple, dim3(1024), dim3(256), 0, st, m.adv_coefs_3rd, (int64_t)(b.d.nEdges + 1) * 15, c3);
    hipLaunchKernelGGL(k_mi_couple, dim3(1024), dim3(256), 0, st, m.zb3_cell,
                       (int64_t)(b.d.nCells + 1) * b.me_decl * (b.d.K + 1), c3);
    hipLaunchKernelGGL(k_mi_mesh_scaling, grid(std::max(b.d.nCells, b.d.nEdges)), dim3(256), 0, st, m,
                       (int)(h_scale_with_mesh != 0));
    hipLaunchKernelGGL(k_mi_damping, grid((int64_t)b.d.nCells * b.d.K), dim3(256), 0, st, m, config_zd, config_xnutr);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->bnd_ready = false;  // signs, zb_cell, zb3_cell, kiteForCell changed: pack_mesh and the records again
  return MPAS_DYC_OK;
}

int mpas_dyc_init_deriv_two(mpas_dyc_ctx* ctx, int32_t block, const double* xp, const double* yp,
                            const double* sin_the, const double* cos_the) {
  if (!ctx || !xp || !yp || !sin_the || !cos_the) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  if (block < 0 || block >= (int)ctx->blk.size()) {
    ctx->err = "mpas_dyc_init_deriv_two: no block " + std::to_string(block);
    return MPAS_DYC_EINVAL;
  }
  Block& b = ctx->blk[block];
  HIPCHK(hipSetDevice(ctx->device));
  Field* f = find(b, "mesh", "deriv_two");
  const int64_t nb = field_bytes(b, *f);
  if (!f->buf[0]) HIPCHK(hipMalloc(&f->buf[0], nb + 256));
  const size_t n = (size_t)b.d.nCells * b.me_decl;
  double* in = nullptr;
  int* bad = nullptr;
  HIPCHK(hipMalloc(&in, 4 * n * sizeof(double) + 256));
  auto run = [&]() -> hipError_t {
    hipError_t e = hipMalloc(&bad, sizeof(int));
    const double* src[4] = {xp, yp, sin_the, cos_the};
    for (int i = 0; i < 4 && e == hipSuccess; ++i)
      e = hipMemcpyAsync(in + i * n, src[i], n * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(f->buf[0], 0, nb, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(bad, 0, sizeof(int), ctx->stream);
    if (e != hipSuccess) return e;
    D2Fit q{};
    q.nEdgesOnCell = (const int*)find(b, "mesh", "nEdgesOnCell")->buf[0];
    q.edgesOnCell = (const int*)find(b, "mesh", "edgesOnCell")->buf[0];
    q.cellsOnEdge = (const int*)find(b, "mesh", "cellsOnEdge")->buf[0];
    q.xp = in;
    q.yp = in + n;
    q.sin_the = in + 2 * n;
    q.cos_the = in + 3 * n;
    q.deriv_two = (double*)f->buf[0];
    q.bad = bad;
    q.nCells = b.d.nCells;
    q.nEdges = b.d.nEdges;
    q.maxEdges = b.me_decl;
    hipLaunchKernelGGL(k_mi_deriv_two, dim3((unsigned)((b.d.nCells + 127) / 128)), dim3(128), 0, ctx->stream, q);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e;
  };
  const hipError_t e = run();
  int hbad = 0;
  if (e == hipSuccess && bad) (void)hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost);
  (void)hipFree(in);
  if (bad) (void)hipFree(bad);
  if (e != hipSuccess) {
    ctx->err = std::string("mpas_dyc_init_deriv_two: ") + hipGetErrorString(e);
    return MPAS_DYC_EHIP;
  }
  if (hbad) {
    ctx->err = "mpas_dyc_init_deriv_two: a cell has more than 14 edges (deriv_two holds 15 weights per side)";
    return MPAS_DYC_EINVAL;
  }
  return MPAS_DYC_OK;
}

int mpas_dyc_init_zb(mpas_dyc_ctx* ctx, int32_t block, int32_t theta_adv_order) {
  if (!ctx || theta_adv_order < 2 || theta_adv_order > 4) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  if (block < 0 || block >= (int)ctx->blk.size()) {
    ctx->err = "mpas_dyc_init_zb: no block " + std::to_string(block);
    return MPAS_DYC_EINVAL;
  }
  Block& b = ctx->blk[block];
  for (const char* n : {"deriv_two", "areaCell"})
    if (!find(b, "mesh", n)->buf[0]) {
      ctx->err = std::string("mpas_dyc_init_zb needs mesh.") + n + " (set it or compute it first)";
      return MPAS_DYC_ESTATE;
    }
  HIPCHK(hipSetDevice(ctx->device));
  ZbFit q{};
  for (const char* n : {"zb", "zb3"}) {
    Field* f = find(b, "mesh", n);
    const int64_t nb = field_bytes(b, *f);
    if (!f->buf[0]) HIPCHK(hipMalloc(&f->buf[0], nb + 256));
    HIPCHK(hipMemsetAsync(f->buf[0], 0, nb, ctx->stream));
    (n[2] ? q.zb3 : q.zb) = (double*)f->buf[0];
  }
  q.nEdgesOnCell = (const int*)find(b, "mesh", "nEdgesOnCell")->buf[0];
  q.cellsOnCell = (const int*)find(b, "mesh", "cellsOnCell")->buf[0];
  q.cellsOnEdge = (const int*)find(b, "mesh", "cellsOnEdge")->buf[0];
  q.deriv_two = (const double*)find(b, "mesh", "deriv_two")->buf[0];
  q.zgrid = (const double*)find(b, "mesh", "zgrid")->buf[0];
  q.dcEdge = (const double*)find(b, "mesh", "dcEdge")->buf[0];
  q.dvEdge = (const double*)find(b, "mesh", "dvEdge")->buf[0];
  q.areaCell = (const double*)find(b, "mesh", "areaCell")->buf[0];
  q.nCells = b.d.nCells;
  q.nCellsSolve = b.d.nCellsSolve;
  q.nEdges = b.d.nEdges;
  q.K = b.d.K;
  q.maxEdges = b.me_decl;
  q.order = theta_adv_order;
  const int64_t n = (int64_t)b.d.nEdges * b.d.K;
  hipLaunchKernelGGL(k_mi_zb, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, q);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->stream));
  ctx->bnd_ready = false;  // zb / zb3 feed model_init's zb_cell copies
  return MPAS_DYC_OK;
}

int mpas_dyc_init_reconstruct(mpas_dyc_ctx* ctx) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  int* bad = nullptr;
  HIPCHK(hipMalloc(&bad, sizeof(int)));
  int rc = MPAS_DYC_OK;
  for (auto& b : ctx->blk) {
    RecInit q{};
    const double* xyz[6];
    const char* names[6] = {"xCell", "yCell", "zCell", "xEdge", "yEdge", "zEdge"};
    for (int i = 0; i < 6; ++i) {
      xyz[i] = (const double*)find(b, "mesh", names[i])->buf[0];
      if (!xyz[i]) {
        ctx->err = std::string("mpas_dyc_init_reconstruct needs mesh.") + names[i] + " (set it first)";
        rc = MPAS_DYC_ESTATE;
      }
    }
    if (rc != MPAS_DYC_OK) break;
    q.nEdgesOnCell = (const int*)find(b, "mesh", "nEdgesOnCell")->buf[0];
    q.edgesOnCell = (const int*)find(b, "mesh", "edgesOnCell")->buf[0];
    q.cellsOnEdge = (const int*)find(b, "mesh", "cellsOnEdge")->buf[0];
    q.xCell = xyz[0];
    q.yCell = xyz[1];
    q.zCell = xyz[2];
    q.xEdge = xyz[3];
    q.yEdge = xyz[4];
    q.zEdge = xyz[5];
    Field* f = find(b, "mesh", "coeffs_reconstruct");
    q.coeffs = (double*)f->buf[0];
    q.bad = bad;
    q.nCells = b.d.nCells;
    q.maxEdges = b.me_decl;
    if (hipMemsetAsync(f->buf[0], 0, field_bytes(b, *f), ctx->stream) != hipSuccess ||
        hipMemsetAsync(bad, 0, sizeof(int), ctx->stream) != hipSuccess) {
      rc = MPAS_DYC_EHIP;
      break;
    }
    hipLaunchKernelGGL(k_mi_reconstruct, dim3((unsigned)((b.d.nCells + 127) / 128)), dim3(128), 0, ctx->stream, q);
    int hbad = 0;
    if (hipGetLastError() != hipSuccess || hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = MPAS_DYC_EHIP;
      break;
    }
    if (hbad) {
      ctx->err = "mpas_dyc_init_reconstruct: a cell has more than 14 edges";
      rc = MPAS_DYC_EINVAL;
      break;
    }
  }
  if (rc == MPAS_DYC_EHIP) ctx->err = "mpas_dyc_init_reconstruct: HIP error";
  (void)hipFree(bad);
  ctx->bnd_ready = false;  // pack_mesh copies coeffs_reconstruct for the kernels
  return rc;
}

int mpas_dyc_output_diagnostics(mpas_dyc_ctx* ctx, int32_t time_level) {
  if (!ctx || (time_level != 1 && time_level != 2)) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  for (auto& b : ctx->blk) {
    const Ptrs p = make_ptrs(ctx, b);
    const Dims& d = b.d;
    LAUNCH(k_output_diagnostics, d.nCells, d, p, (int)time_level, ctx->index_qv);
  }
  HIPCHK(hipGetLastError());
  return MPAS_DYC_OK;
}

int mpas_dyc_timestep(mpas_dyc_ctx* ctx, double dt, int32_t itimestep) {
  (void)itimestep;
  if (!ctx || !(dt > 0.0)) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  CHK(plan_all(ctx, dt));
  ctx->tail_pending = (ctx->physics & MPAS_DYC_PHYSICS_MICROPHYSICS) != 0;
  if (ctx->profile) return profiled_step(ctx, dt);
  if (ctx->use_graph) {
    // one captured graph per buffer layout the step starts from; capturing runs srk3, whose
    // rotations move the host's view of the buffers, and a replay repeats them
    const std::string sig = layout_sig(ctx);
    auto git = ctx->graphs.find(sig);
    if (git == ctx->graphs.end() || ctx->graph_dt[sig] != dt) {
      if (git != ctx->graphs.end() && git->second) (void)hipGraphExecDestroy(git->second);
      ctx->graphs.erase(sig);
      hipGraph_t g = nullptr;
      hipGraphExec_t ge = nullptr;
      const Layout l0 = save_layout(ctx);
      HIPCHK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
      int r = srk3(ctx, dt);
      hipError_t e = hipStreamEndCapture(ctx->stream, &g);
      if (r && r != MPAS_DYC_ECOMM) {  // nothing ran: undo the capture's rotations of the host view
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        restore_layout(l0);
        return r;
      }
      if (r == MPAS_DYC_ECOMM && e == hipSuccess) e = hipErrorUnknown;  // RCCL refused to be captured
      if (e == hipSuccess) e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      if (g) (void)hipGraphDestroy(g);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        restore_layout(l0);  // nothing ran: the eager step below rotates from the start
        if (ctx->nranks > 1) {  // every rank captures or the job fails: no rank goes eager alone
          ctx->err = std::string("hipGraph capture of the step failed on rank ") + std::to_string(ctx->rank) + ": " +
                     hipGetErrorString(e);
          return MPAS_DYC_EHIP;
        }
        // one process: a runtime that cannot capture this step runs it eagerly, and says so
        ctx->use_graph = false;
        ctx->graph_ran = false;
        fprintf(stderr, "mpas_dycore: hipGraph capture failed (%s); running the step eagerly\n",
                hipGetErrorString(e));
        r = srk3(ctx, dt);
        HIPCHK(hipGetLastError());
        return r;
      }
      ctx->graphs[sig] = ge;
      ctx->graph_dt[sig] = dt;
      HIPCHK(hipGraphLaunch(ge, ctx->stream));  // the capture made the step's rotations already
      ctx->graph_ran = true;
      return MPAS_DYC_OK;
    }
    HIPCHK(hipGraphLaunch(git->second, ctx->stream));
    apply_step_rotations(ctx);
    ctx->graph_ran = true;
    return MPAS_DYC_OK;
  }
  ctx->graph_ran = false;
  int r = srk3(ctx, dt);
  HIPCHK(hipGetLastError());
  return r;
}

int mpas_dyc_set_profile(mpas_dyc_ctx* ctx, int32_t on) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  ctx->profile = on != 0;
  return MPAS_DYC_OK;
}

int mpas_dyc_get_profile(mpas_dyc_ctx* ctx, double* out, int32_t n) {
  if (!ctx || !out || n < 1) return MPAS_DYC_EINVAL;
  for (int i = 0; i < n; ++i) out[i] = i < 5 ? ctx->prof_out[i] : 0.0;
  return MPAS_DYC_OK;
}

const char* mpas_dyc_last_exchange(const mpas_dyc_ctx* ctx) { return ctx ? ctx->last_key : ""; }

int32_t mpas_dyc_rccl_version(void) {
  int v = 0;
  return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

int mpas_dyc_finish_step(mpas_dyc_ctx* ctx, double dt) {
  if (!ctx || !(dt > 0.0)) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  if (!(ctx->physics & MPAS_DYC_PHYSICS_MICROPHYSICS)) return MPAS_DYC_OK;  // the step ran its own tail
  HIPCHK(hipSetDevice(ctx->device));
  const std::vector<Ptrs> P = block_ptrs(ctx);
  ctx->tail_pending = false;
  int r = step_tail(ctx, P, dt);
  HIPCHK(hipGetLastError());
  return r;
}

int mpas_dyc_graph_active(const mpas_dyc_ctx* ctx) { return ctx && ctx->graph_ran ? 1 : 0; }

int mpas_dyc_plan_exchanges(mpas_dyc_ctx* ctx, int32_t nranks, int32_t rank, double dt, mpas_dyc_plan_msg* msgs,
                            int64_t cap, int64_t* n_msgs, char* keys, int64_t keys_bytes, int64_t* keys_len) {
  if (!ctx || !n_msgs || !keys_len || nranks < 1 || rank < 0 || rank >= nranks || !(dt > 0.0) || cap < 0 ||
      keys_bytes < 0)
    return MPAS_DYC_EINVAL;
  if (!ctx->host_only) {
    ctx->err = "mpas_dyc_plan_exchanges needs a MPAS_DYC_HOST_ONLY context";
    return MPAS_DYC_ESTATE;
  }
  ctx->nranks = nranks;
  ctx->rank = rank;
  invalidate_plans(ctx);
  std::vector<std::string> seq;
  ctx->record = &seq;
  ctx->planning = true;
  const int cur0 = ctx->cur;
  const Layout l0 = save_layout(ctx);
  int r = init_diagnostics(ctx, dt);
  for (int step = 0; step < 2 && r == MPAS_DYC_OK; ++step) {
    r = srk3(ctx, dt);
    ctx->cur ^= 1;  // mpas_dyc_shift_time_levels
  }
  ctx->cur = cur0;
  restore_layout(l0);
  ctx->planning = false;
  ctx->record = nullptr;
  if (r) return r;
  int64_t nm = 0, kl = 1;
  for (size_t i = 0; i < seq.size(); ++i) {
    const XPlan& pl = ctx->plans.at(seq[i]);
    for (int dir = 0; dir < 2; ++dir)
      for (const XMsg& m : dir == 0 ? pl.rsend : pl.rrecv) {
        if (msgs && nm < cap)
          msgs[nm] = mpas_dyc_plan_msg{(int32_t)i, dir == 0 ? MPAS_DYC_SEND : MPAS_DYC_RECV, m.block, m.peer_rank,
                                       m.peer_block, m.count};
        ++nm;
      }
    kl += (int64_t)seq[i].size() + 1;
  }
  *n_msgs = nm;
  *keys_len = kl;
  if (keys && kl <= keys_bytes) {
    char* q = keys;
    for (const auto& k : seq) {
      memcpy(q, k.data(), k.size());
      q += k.size();
      *q++ = '\n';
    }
    *q = '\0';
  }
  return (nm > cap || kl > keys_bytes) ? MPAS_DYC_EINVAL : MPAS_DYC_OK;
}

int mpas_dyc_shift_time_levels(mpas_dyc_ctx* ctx) {
  if (!ctx) return MPAS_DYC_EINVAL;
  ctx->cur ^= 1;
  return MPAS_DYC_OK;
}

int mpas_dyc_synchronize(mpas_dyc_ctx* ctx) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->xstream));
  return p2p_check(ctx);
}

int mpas_dyc_set_p2p(mpas_dyc_ctx* ctx, int32_t on) {
  if (!ctx) return MPAS_DYC_EINVAL;
  if (on < 0) return MPAS_DYC_OK;  // keep what the environment chose at creation
  invalidate_plans(ctx);
  ctx->p2p = on != 0;
  return MPAS_DYC_OK;
}

int mpas_dyc_get_p2p(const mpas_dyc_ctx* ctx) { return ctx && ctx->p2p ? 1 : 0; }

int mpas_dyc_set_overlap(mpas_dyc_ctx* ctx, int32_t on) {
  if (!ctx) return MPAS_DYC_EINVAL;
  invalidate_plans(ctx);
  ctx->overlap = on < 0 ? -1 : (on != 0);
  return MPAS_DYC_OK;
}

int mpas_dyc_use_graph(mpas_dyc_ctx* ctx, int32_t on) {
  if (!ctx) return MPAS_DYC_EINVAL;
  ctx->use_graph = on != 0;
  return MPAS_DYC_OK;
}

int mpas_dyc_block_layout(mpas_dyc_ctx* ctx, int32_t block, int32_t* out) {
  Block* b = get_block(ctx, block);
  if (!b || !out) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->bnd_ready) CHK(compute_bnd(ctx));
  out[0] = b->d.maxEdges;
  out[1] = b->d.maxEdges2;
  out[2] = pair_layout(b->d) ? 2 : batched(b->d) ? 1 : 0;
#ifdef MPAS_WIDE
  out[3] = WIDE_THREADS == 128 ? 1 : WIDE_THREADS == 256 ? 2 : 3;
#else
  out[3] = 0;
#endif
  return MPAS_DYC_OK;
}

double mpas_dyc_acoustic_bytes(const mpas_dyc_ctx* ctx) {
  if (!ctx) return 0.0;
  // B_ac = 8 [K (7 nE_act + 18 nC_own) + 9 (K+1) nC_own]   (SURVEY.md §8d), block 0
  const Dims& d = ctx->blk[0].d;
  const double K = d.K;
  const double nEact = ctx->blk[0].nEdges_act >= 0 ? (double)ctx->blk[0].nEdges_act : (double)d.nEdges;
  const double nC = d.nCellsSolve;
  return 8.0 * (K * (7.0 * nEact + 18.0 * nC) + 9.0 * (K + 1.0) * nC);
}

int mpas_dyc_time_acoustic_step(mpas_dyc_ctx* ctx, double dts, int32_t small_step, int32_t reps, double* ms_out,
                                double* ms_kernels) {
  if (!ctx || reps < 1) return MPAS_DYC_EINVAL;
  if (ctx->host_only) return MPAS_DYC_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->bnd_ready) CHK(compute_bnd(ctx));
  Block& b = ctx->blk[0];
  const Ptrs p = make_ptrs(ctx, b);
  const Dims& d = b.d;
  // the sequence srk3 runs for a `reps`-sub-step acoustic loop: edges, cells, then per further
  // sub-step the damped edge phase and cells, and the last sub-step's damping on its own.  One
  // event between consecutive launches, read after the loop: the kernels run back to back as in
  // srk3, and no host launch latency after an idle queue lands inside a kernel's interval.
  // The events carry no system-scope fence (hipEventDisableSystemFence): a default event between
  // two kernels writes back and invalidates L2, so every timed kernel would start on a cold cache,
  // which srk3's captured step never does (measured: the loop's kernels ran 10-20 % longer than the
  // same kernels inside the step).  The stream is synchronised before the events are read.
  double acc[3] = {0, 0, 0};
  float t;
  std::vector<hipEvent_t> ev(2 * (size_t)reps + 2);  // + the end of the damping
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  auto destroy = [&]() {
    for (auto& e : ev) (void)hipEventDestroy(e);
  };
  HIPCHK(hipEventRecord(ev[0], ctx->stream));
  for (int r = 0; r < reps; ++r) {
    acoustic_edges(ctx, d, p, dts, small_step, r > 0 ? 1 : 0, 0);
    HIPCHK(hipEventRecord(ev[2 * r + 1], ctx->stream));
    acoustic_cells(ctx, d, p, dts, small_step);
    HIPCHK(hipEventRecord(ev[2 * r + 2], ctx->stream));
  }
  divergence_damping(ctx, d, p, dts, 0);
  const size_t e_end = 2 * (size_t)reps + 1;
  HIPCHK(hipEventRecord(ev[e_end], ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  (void)hipEventElapsedTime(&t, ev[2 * (size_t)reps], ev[e_end]);
  acc[2] += t;
  for (int r = 0; ms_kernels && r < reps; ++r) {
    (void)hipEventElapsedTime(&t, ev[2 * r], ev[2 * r + 1]);
    acc[0] += t;
    (void)hipEventElapsedTime(&t, ev[2 * r + 1], ev[2 * r + 2]);
    acc[1] += t;
  }
  float tot;
  (void)hipEventElapsedTime(&tot, ev[0], ev[e_end]);
  destroy();
  if (ms_out) *ms_out = tot / reps;
  if (ms_kernels)
    for (int i = 0; i < 3; ++i) ms_kernels[i] = acc[i] / reps;
  return MPAS_DYC_OK;
}

}  // extern "C"
