// SDFS shared pieces: RPC method ids, storage naming, path specs, the
// get-versions merge format, and the leader's replica-placement rule.
//
// Reference: storage_filename = sanitize("v{version}." + filename)
// (src/services.rs:550-552); merge_versions writes "{:=^40}" version
// delimiters in descending version order (src/services.rs:554-569); new
// replicas are chosen as (hash(filename) + i) % n over the active non-replica
// ids (src/services.rs:346-364).
#pragma once
#include <cstdint>
#include <set>
#include <string>
#include <vector>

#include "membership.h"

namespace dmlc {
namespace ctl {

// Port layout per node, matching the reference's 8850/8851/8852 triple:
// membership UDP = base, leader RPC = base+1, member RPC = base+2.
inline int leader_port(int base) { return base + 1; }
inline int member_port(int base) { return base + 2; }

enum LeaderMethod : uint16_t {
  L_GET = 1,
  L_GET_VERSIONS = 2,
  L_PUT = 3,
  L_DELETE = 4,
  L_LS = 5,
  L_TRAIN = 6,
  L_PREDICT = 7,  // payload: optional u32 count + SDFS shard names (jobs over shards)
  L_JOBS = 8,
  L_ALIVE = 9,
  L_STATE = 10,  // jobs + SDFS directory snapshot (standby replication)
  L_PREDICT_SHARD = 11,  // classify an SDFS u8 shard on a replica holder (HBM-resident)
};

enum MemberMethod : uint16_t {
  M_GET_LATEST_VERSION = 20,
  M_RECEIVE = 21,
  M_PREDICT = 22,
  M_FETCH = 23,       // pull a file from another member (third-party copy)
  M_READ_CHUNK = 24,  // serve a byte range of a local file
  M_DELETE_FILE = 25,
  M_LOAD_MODEL = 26,  // hot-swap model weights (train)
  M_INFO = 27,
  M_PREDICT_SHARD = 28,  // classify the local (HBM-staged) replica of a shard
  M_SHARD_INFO = 29,     // header of the local replica of a shard (n, h, w, labels)
  M_PREDICT_RANGE = 30,  // classify images [first, first+n) of the local replica of a shard
};

std::string sanitize_filename(const std::string& s);
std::string storage_filename(const std::string& filename, int version);
// "{:=^40}" of " Version N " (Rust centre alignment: extra pad on the right).
std::string version_delimiter(int version);
// Merge fetched v{n}.<basename> files next to `dest` into `dest`.
void merge_versions(const std::string& dest, const std::set<int>& versions);
std::string versioned_sibling(const std::string& dest, int version);  // dir/v{n}.{basename}

// Deterministic placement: up to `need` ids from `candidates` (ascending).
std::set<Id> choose_replicas(const std::string& filename, const std::vector<Id>& candidates, int need);

using Directory = std::map<std::string, std::map<Id, std::set<int>>>;
void write_directory(Writer& w, const Directory& d);
Directory read_directory(Reader& r);

}  // namespace ctl
}  // namespace dmlc
