// Ring-heartbeat membership list and failure detector (SWIM-like, full-list
// gossip piggybacked on pings).
//
// Reference: src/membership.rs (MembershipService::run/join/leave/
// list_membership/list_self/id/active_ids :66-148, receiver :150-223, pinger
// :225-259, detector :261-291, LWW merge with Failed-wins ties :302-327).
// Behaviour kept: Id = (address, incarnation timestamp); every period each
// node refreshes its own last_active and pings <= 2k ring neighbours (k = 2)
// with its whole list; receivers merge (last-writer-wins on last_active, a
// tie goes to Failed), ack, and the detector marks a last-round neighbour
// Failed when its last_active is older than the timeout. Join goes through an
// introducer that fails older incarnations of the same address and answers
// Welcome with the full list.
// Fixed reference quirks: `leave` also tells the ring
// neighbours (Leave message) instead of only clearing the list (#1); Failed
// tombstones are garbage-collected after `tombstone_ms` and GC'd ids are not
// re-admitted (#2); datagrams up to 64 KB (#2); every port, period and
// timeout is configurable (#9). Failure detection no longer compares a remote
// wall-clock stamp with the local clock (#3): last_active still orders one
// node's own heartbeats (LWW), but the detector and tombstone GC age an entry
// by the LOCAL steady time at which its last_active last advanced (heard_),
// so clock skew between nodes cannot fail a live node (`--clock-skew-ms`
// injects skew for the test). Fault-injection hooks (drop rate, pause,
// partition) make failure tests deterministic on one machine.
#pragma once
#include <atomic>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "net.h"
#include "wire.h"

namespace dmlc {
namespace ctl {

struct Id {
  std::string address;  // "host:port" of the membership endpoint
  int64_t timestamp = 0;  // incarnation (wall-clock us at join)
  bool operator<(const Id& o) const {
    return address != o.address ? address < o.address : timestamp < o.timestamp;
  }
  bool operator==(const Id& o) const { return address == o.address && timestamp == o.timestamp; }
  bool operator!=(const Id& o) const { return !(*this == o); }
  std::string host() const;
  int port() const;
  std::string debug() const;  // Id { address: "...", timestamp: ... }
};

enum class Status : uint8_t { Active = 0, Failed = 1 };
const char* status_name(Status s);

struct Membership {
  Status status = Status::Active;
  int64_t last_active = 0;  // wall-clock us
  bool operator==(const Membership& o) const { return status == o.status && last_active == o.last_active; }
};

using MembershipList = std::map<Id, Membership>;

enum class MsgType : uint8_t { Ping = 1, Ack = 2, Join = 3, Welcome = 4, Leave = 5 };

struct Message {
  MsgType type;
  Id sender;
  int64_t last_active = 0;  // Ack
  MembershipList list;      // Ping, Welcome
};

std::string encode_message(const Message& m);
Message decode_message(const char* p, size_t n);
void write_id(Writer& w, const Id& id);
Id read_id(Reader& r);

// Merge rule (pure, unit-tested): returns true if anything changed. No-op
// when `local` is empty (not joined / left). Ids in `dead` are ignored.
bool merge_membership(MembershipList& local, const MembershipList& remote,
                      const std::set<Id>& dead = {},
                      std::vector<std::string>* status_changes = nullptr);

struct MembershipConfig {
  std::string bind_host = "0.0.0.0";
  std::string host = "127.0.0.1";  // advertised
  int port = 8850;
  int ping_ms = 1000;
  int detect_ms = 1000;
  int fail_ms = 3000;
  int tombstone_ms = 30000;
  int k = 2;
  int64_t clock_skew_us = 0;  // fault injection: offset on this node's own wall clock
};

class MembershipService {
 public:
  explicit MembershipService(MembershipConfig cfg);
  ~MembershipService();
  void start();
  void stop();

  // CLI verbs
  void join(const std::string& introducer);  // "host:port"
  void leave();
  MembershipList snapshot() const;
  Id id() const;
  std::set<Id> active_ids() const;
  std::vector<Id> active_sorted() const;
  std::vector<Id> neighbors() const;

  // fault injection
  void set_drop_rate(double p) { drop_rate_ = p; }
  void set_paused(bool p) { paused_ = p; }
  void partition(const std::string& addr);
  void heal();

  // counters
  uint64_t sent() const { return sent_; }
  uint64_t received() const { return received_; }

 private:
  void receiver_loop();
  void pinger_loop();
  void detector_loop();
  void send(const std::string& addr, const Message& m);
  bool blocked(const std::string& addr);
  void note_heard_locked();  // refresh heard_ from list_ (mu_ held)
  int64_t own_us() const { return wall_us() + cfg_.clock_skew_us; }

  MembershipConfig cfg_;
  mutable std::mutex mu_;
  MembershipList list_;
  Id id_;
  std::set<Id> dead_;  // GC'd tombstones
  std::vector<Id> last_neighbors_;
  Fd sock_;
  std::atomic<bool> stop_{false};
  std::thread rx_, ping_, det_;
  std::atomic<double> drop_rate_{0.0};
  std::atomic<bool> paused_{false};
  std::mutex part_mu_;
  std::set<std::string> partitioned_;
  std::mutex rng_mu_;
  std::mt19937_64 rng_{std::random_device{}()};
  std::atomic<uint64_t> sent_{0}, received_{0};
  // id -> (newest last_active seen, local steady us when it last advanced)
  std::map<Id, std::pair<int64_t, int64_t>> heard_;
};

}  // namespace ctl
}  // namespace dmlc
