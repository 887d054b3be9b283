// Engine object behind the C ABI.
#pragma once
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "exprc.h"
#include "nbg_internal.h"

namespace nbg {

struct Engine {
  nbg_config cfg{};
  std::string last_error;
  std::map<int32_t, SchemaSet> edges;   // positive edge types
  std::map<int32_t, SchemaSet> tags;
  // staging (until finalize)
  std::map<int32_t, EdgeStage> stage;   // signed type -> records
  std::map<int32_t, TagStage> tstage;   // tag id -> vertex records
  std::vector<std::string> pool;        // string props, load order
  std::unordered_map<std::string, int64_t> pool_index;
  uint64_t seq = 0;
  bool finalized = false;
  // device
  Snapshot snap;
  hipStream_t stream = nullptr;
  Workspace* ws = nullptr;
  std::mutex mu;
  // asynchronous GO (nbg_go_submit / nbg_go_wait): query slots, each a workspace on its own stream
  struct QuerySlot {
    Workspace* ws = nullptr;
    hipStream_t stream = nullptr;
    void* ticket = nullptr;   // the ticket running on this slot (nullptr: free)
    // partitioned engine: the slot's own communicator (split from `comm` when the slot is first
    // used) lets its queries run on its own stream beside the other slots'
    std::unique_ptr<Comm> comm;
    bool comm_tried = false;
  };
  std::vector<QuerySlot> slots;
  SpCtx* sp = nullptr;                  // one-pair FIND SHORTEST PATH workspace (sp.hip), on `stream`
  struct PathSlot {                     // asynchronous FIND SHORTEST PATH (nbg_find_path_submit)
    SpCtx* sp = nullptr;
    hipStream_t stream = nullptr;
    void* ticket = nullptr;
  };
  std::vector<PathSlot> path_slots;
  std::vector<void*> path_inflight;
  // nbg_find_path_batch: one-pair SHORTEST queries run NBG_SP_BATCH at a time as one batched
  // launch chain, on workspaces sharing one stream
  std::vector<SpCtx*> batch_sp;
  bool batch_sp_full = false;     // the last growth stopped at the HBM reserve (nbg_path_reserve retries)
  unsigned long long batch_reruns = 0;   // batched pairs rerun on `sp` after a list overflow
  hipStream_t batch_stream = nullptr;
  uint64_t max_dict_len = 0;            // the longest dictionary string (derived-string arena bound),
  uint64_t max_dict_len_of = ~0ull;     //   computed for a dictionary of this many strings
  uint64_t row_reserve = 0;             // result rows of the largest prepared GO statement (new
  int col_reserve = 0;                  // query workspaces are sized for it before their first query)
  int prof_mode = 0;
  // pinned host blocks of fetched GO rows (nbg_rows_fetch), reused across queries
  std::mutex pinned_mu;
  std::vector<std::pair<size_t, void*>> pinned_free;
  void* pinned_get(size_t bytes, size_t* got);
  void pinned_put(void* p, size_t bytes);
  void pinned_release();                    // nbg_profile mode (applied to shortest-path contexts made later)
  SpCtx* new_sp(hipStream_t s, std::string* err);   // sp_create for this snapshot + the profile mode
  uint64_t sp_item_cap() const;         // items a shortest-path list may hold
  uint64_t sp_edge_cap() const;         // edges of the larger direction (a level's edge space)
  std::vector<void*> inflight;          // submitted tickets, oldest first
  // device GO results (rows left in HBM) and the workspace their rows live in: before that
  // workspace runs another query it is handed to the result (freed with it) and replaced
  std::unordered_map<Workspace*, ::nbg_rows*> holders;
  // multi-GPU (partitioned mode when cfg.num_gpus > 1): global id = owner * npad + local id
  std::unique_ptr<Comm> comm;
  uint64_t npad = 0;
  bool partitioned() const { return cfg.num_gpus > 1; }
  // partitioned: every rank's dictionary (global id order) and every vertex's out-degree per positive
  // type over the global id space, host copies from finalize, so that every rank bounds a GO first
  // hop's edges per owner alike (go_launch sends a small hop as slot arrays instead of bitmaps)
  std::vector<int64_t> h_gdict;
  std::vector<uint64_t> h_gcount;
  std::map<int32_t, std::vector<uint32_t>> h_gdeg;
  int32_t gather_degrees();   // (collective, at finalize)
  // the most edges (capped degrees) the starts hold on any one rank; UINT64_MAX when unknown
  uint64_t first_hop_bound(int32_t type, const int64_t* starts, uint64_t n, uint32_t cap) const;

  // FIND PATH replica of a partitioned snapshot (replica.hip): a single-GPU engine over every
  // rank's path CSRs; FIND PATH runs on it rank-locally while it is in use
  std::unique_ptr<Engine> rep;
  // partitioned GO: what a rank whose query preparation failed takes part in the query's
  // collectives with (go_launch): a zero send bitmap, a receive scratch, the statistics words
  void* fb_send = nullptr;
  void* fb_recv = nullptr;
  unsigned long long* fb_gst = nullptr;
  unsigned long long* fb_hgst = nullptr;
  int path_replica_mode = -1;   // build it at finalize: 1 yes (when it fits), 0 no, -1 NBG_PATH_REPLICA (default 1)
  std::atomic<bool> path_replica_use{true};   // nbg_set_path_replica after finalize: 0 = the collective search
  Engine* path_engine() { return rep && path_replica_use.load() ? rep.get() : this; }
  // the replica's failures are reported through its parent's nbg_last_error too
  Engine* err_parent = nullptr;
  std::mutex err_mu;

  uint64_t tiny_queries = 0;    // GO queries run by ws_go_tiny (nbg_stats)
  uint64_t host_agreements = 0; // partitioned GO queries that agreed on the host first (nbg_stats)
  // nbg_inject_fault (tests): the next fault_count queries fail at fault_site
  int fault_site = 0, fault_count = 0;
  bool fault(int site) {
    if (fault_site != site || fault_count <= 0) return false;
    if (--fault_count == 0) fault_site = 0;
    return true;
  }
  int32_t fail(int32_t code, const std::string& msg) {
    {
      std::lock_guard<std::mutex> lg(err_mu);
      last_error = msg;
    }
    if (err_parent) {
      std::lock_guard<std::mutex> lg(err_parent->err_mu);
      err_parent->last_error = msg;
    }
    return code;
  }
  int64_t intern(const std::string& s);
  bool decode_row(const SchemaSet& ss, const uint8_t* v, size_t n, int64_t* out);
  int32_t load_part_kv(int32_t part, const uint8_t* kd, const uint64_t* ko, const uint8_t* vd, const uint64_t* vo,
                       uint64_t n);
  // SST-file ingest (sst.cpp): one file into one part / NebulaStore::ingest over download/<part>
  int32_t ingest_sst(int32_t part, const std::string& path);
  int32_t ingest_dir(const std::string& download);
  int32_t load_edges(int32_t type, const int64_t* src, const int64_t* dst, const int64_t* rank, uint64_t n,
                     const void* const* cols, int32_t ncols);
  int32_t finalize();
  int32_t build_tags(const std::vector<int64_t>& dict, const std::vector<int64_t>& remap);
  int32_t upload_tags();   // DevTag host arrays -> device (+ all-gather when partitioned)
  bool upload_type(DevEdgeType& dt, uint64_t nv, const std::vector<uint32_t>& col, const std::vector<int64_t>& dvid,
                   const std::vector<int64_t>* rk, const std::vector<std::vector<int64_t>>& pc,
                   const std::vector<uint8_t>* valid, const std::vector<VKind>& kinds);
  int32_t upload_vertices(const std::vector<uint8_t>& visible, bool all_visible);
  int32_t save_snapshot(const char* path);
  int32_t load_snapshot(const char* path);
  // partitioned: the union of every rank's sorted string set (one dictionary, so string codes
  // mean the same on every rank: gathered $$ columns, rows exchanged for DISTINCT)
  int32_t exchange_strings(std::vector<std::string>* strings);
  int32_t exchange_dictionary(const std::vector<int64_t>& local, std::vector<int64_t>* gdict,
                              std::vector<uint64_t>* gcount);
  uint32_t dense(int64_t vid) const;
  void free_snapshot();   // release every device array of `snap` and reset it
  int32_t upload_strings();         // the dictionary's device tables (engine_ready)
  DevStrings dev_strings() const;   // ... as the kernels read them (no arena)
};

int32_t engine_ready(Engine& E);   // workspace (+ partition buffers) after finalize / snapshot load
// replica.hip: the FIND PATH replica of a partitioned engine (collective; no replica when it does
// not fit, is not wanted, or a vertex sits on two ranks)
int32_t build_path_replica(Engine& E);
void destroy_path_replica(Engine& E);
bool path_replica_wanted(const Engine& E);
void path_slots_release(Engine& E); // completes outstanding path tickets, frees the path slots
// Make *wsp free for a new query: if live device rows still sit in it, the rows take the
// workspace over and *wsp becomes a fresh one on `stream` (profiling state carried over).
int32_t ws_release(Engine& E, Workspace** wsp, hipStream_t stream);

}  // namespace nbg

struct nbg_engine {
  nbg::Engine e;
};

struct nbg_paths {
  std::vector<std::vector<int64_t>> paths;
  uint64_t edges = 0;   // BFS adjacency entries scanned, both directions
  uint32_t batches = 0; // device chain: launch batches the host enqueued (1: none continued; 0: host loop)
};
