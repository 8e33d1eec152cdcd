// Member service: replica registry, SDFS data plane, inference, leader
// pointer.
//
// Reference: tarpc `Member` (get_latest_version / receive / predict,
// src/services.rs:443-497), MemberState::shared (storage wipe, model load,
// leader health loop, src/services.rs:502-548), check_leader
// (src/services.rs:571-580). Differences: bulk data moves member-to-member
// over this RPC (M_FETCH pulls chunks with M_READ_CHUNK) instead of `scp`;
// `delete` removes replica files; `train` hot-swaps weights (M_LOAD_MODEL);
// the leader pointer wraps around the candidate list.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../serve/executor.h"
#include "../serve/shard.h"
#include "membership.h"
#include "rpc.h"
#include "sdfs.h"

namespace dmlc {
namespace ctl {

struct MemberConfig {
  std::string bind_host = "0.0.0.0";
  std::string workdir = ".";
  std::string storage_dir;  // default <workdir>/storage
  std::string models_dir;   // default <workdir>/models
  std::string dataset_dir;  // imagenet_1k/train layout: <dir>/<wnid>/<file>.JPEG
  std::vector<std::string> leader_candidates;  // base addresses "host:port", in order
  int check_ms = 3000;
  // leader heartbeat: an L_ALIVE probe of the current leader every watch_ms
  // (timeout 3 x watch_ms); a closed connection or a missed probe wakes the
  // leader check at once (0: off, the periodic check alone)
  int watch_ms = 250;
  int chunk_bytes = 8 << 20;
  bool hbm_replicas = true;  // stage received u8-shard replicas into the executor's blob store (HBM)
};

// Label table: synset_words.txt lines "<wnid> <label text>" (src/services.rs:170-184).
struct Labels {
  std::vector<std::pair<std::string, std::string>> entries;
  std::map<std::string, int> index;
  static Labels load(const std::string& path);
  std::string text(int idx) const;
};

class MemberService {
 public:
  MemberService(MemberConfig cfg, MembershipService* ms, std::unique_ptr<Executor> exec, Labels labels);
  ~MemberService();
  void start(int base_port);
  void stop();

  std::string leader_address() const;  // base address of the current leader
  std::map<std::string, std::set<int>> files() const;
  std::string resolve_spec(const std::string& spec) const;
  Executor* executor() { return exec_.get(); }
  const Labels& labels() const { return labels_; }

  // local implementations (also reachable over RPC)
  std::vector<std::pair<double, std::string>> predict(const std::string& model, const std::vector<std::string>& ids,
                                                      bool* ok);
  bool fetch(const std::string& src_host, int src_port, const std::string& src_spec, const std::string& dest_spec);

  // What peers may touch through M_READ_CHUNK / M_FETCH / M_LOAD_MODEL:
  // `storage:` and `models:` specs always; an absolute path only while this
  // node's own command that needs it runs — the source of a `put`
  // (readable), the destination of a `get` / `get-versions` (writable, plus
  // its v<N>.<name> siblings). Everything else is refused, so a peer cannot
  // read or write arbitrary files.
  void allow_read(const std::string& abs_path, bool on);
  void allow_write(const std::string& abs_path, bool on);
  std::string readable_path(const std::string& spec) const;  // throws if refused
  std::string writable_path(const std::string& spec) const;  // throws if refused

  // Stage the dataset's query images (first file of every class directory,
  // in label order) into the executor's cache on a background thread, so
  // queries hit HBM-resident images. Returns false if the executor has no
  // cache or a prefetch is already running.
  bool start_prefetch();
  int prefetched() const { return prefetched_.load(); }

  // Classify the local replica (latest version) of SDFS shard `file` from
  // the executor's blob store, staging it first if needed. Returns the
  // version, blob location and per-image predictions.
  struct ShardResult {
    int version = 0;
    std::string location;
    int64_t elapsed_us = 0;
    std::vector<Prediction> preds;
  };
  ShardResult predict_shard(const std::string& file, const std::string& model);
  // Header of the local replica (latest version) of shard `file`; recorded
  // when the replica is staged, so it survives the file's removal from disk.
  struct ShardMeta {
    int version = 0;
    ShardInfo info;
  };
  ShardMeta shard_meta(const std::string& file);
  // Images [first, first + n) of the local replica of `file` (a shard job's
  // query, csrc/serve/leader.cpp): read in place from the executor's blob.
  std::vector<Prediction> predict_range(const std::string& file, const std::string& model, int64_t first, int64_t n);
  // Keys of the staged replicas ("<file>@v<version>").
  std::vector<std::string> staged_replicas() const;

 private:
  std::string query_image(const std::string& id) const;
  void register_handlers();
  void leader_check_loop();
  void leader_watch_loop();
  bool check_leader(const std::string& addr, int timeout_ms = 2000);

  MemberConfig cfg_;
  MembershipService* ms_;
  std::unique_ptr<Executor> exec_;
  Labels labels_;
  std::unique_ptr<RpcServer> server_;
  mutable std::mutex mu_;
  std::map<std::string, std::set<int>> files_;
  std::map<std::string, ShardMeta> shard_meta_;  // under mu_
  std::multiset<std::string> readable_, writable_;  // under mu_
  std::string leader_;
  std::atomic<bool> stop_{false};
  std::thread checker_;
  // Leader watch: a heartbeat to the current leader (MemberConfig::watch_ms)
  // whose failure (the leader's process died: its connections close; or it
  // hangs: probes time out with the sockets still open) wakes the checker at
  // once instead of at its next period.
  std::thread watcher_;
  std::mutex wake_mu_;
  std::condition_variable wake_cv_;
  bool wake_ = false;  // under wake_mu_
  std::thread prefetcher_;
  std::atomic<bool> prefetching_{false};
  std::atomic<int> prefetched_{0};
  // replica staging (received shards -> executor blobs) off the RPC thread
  void replica_loop();
  void stage_replica(const std::string& file, int version);
  std::mutex rq_mu_;
  std::condition_variable rq_cv_;
  std::deque<std::pair<std::string, int>> rq_;
  std::thread replicator_;
};

}  // namespace ctl
}  // namespace dmlc
