#include "membership.h"

#include "common.h"
#include "ring.h"
#include "table.h"

namespace dmlc {
namespace ctl {

std::string Id::host() const { return host_of(address); }
int Id::port() const { return port_of(address); }
std::string Id::debug() const {
  return "Id { address: \"" + address + "\", timestamp: " + format_time_us(timestamp) + " }";
}

const char* status_name(Status s) { return s == Status::Active ? "Active" : "Failed"; }

void write_id(Writer& w, const Id& id) {
  w.str(id.address);
  w.i64(id.timestamp);
}

Id read_id(Reader& r) {
  Id id;
  id.address = r.str();
  id.timestamp = r.i64();
  return id;
}

static void write_list(Writer& w, const MembershipList& l) {
  w.u32((uint32_t)l.size());
  for (const auto& kv : l) {
    write_id(w, kv.first);
    w.u8((uint8_t)kv.second.status);
    w.i64(kv.second.last_active);
  }
}

static MembershipList read_list(Reader& r) {
  MembershipList l;
  uint32_t n = r.u32();
  for (uint32_t i = 0; i < n; ++i) {
    Id id = read_id(r);
    Membership m;
    uint8_t st = r.u8();
    if (st > 1) throw WireError("bad status");
    m.status = (Status)st;
    m.last_active = r.i64();
    l[id] = m;
  }
  return l;
}

std::string encode_message(const Message& m) {
  Writer w;
  w.u8(0xD3);  // magic
  w.u8((uint8_t)m.type);
  write_id(w, m.sender);
  switch (m.type) {
    case MsgType::Ping:
    case MsgType::Welcome:
      write_list(w, m.list);
      break;
    case MsgType::Ack:
    case MsgType::Leave:
      w.i64(m.last_active);
      break;
    case MsgType::Join:
      break;
  }
  return w.take();
}

Message decode_message(const char* p, size_t n) {
  Reader r(p, n);
  if (r.u8() != 0xD3) throw WireError("bad magic");
  Message m;
  uint8_t t = r.u8();
  if (t < 1 || t > 5) throw WireError("bad message type");
  m.type = (MsgType)t;
  m.sender = read_id(r);
  switch (m.type) {
    case MsgType::Ping:
    case MsgType::Welcome:
      m.list = read_list(r);
      break;
    case MsgType::Ack:
    case MsgType::Leave:
      m.last_active = r.i64();
      break;
    case MsgType::Join:
      break;
  }
  return m;
}

bool merge_membership(MembershipList& local, const MembershipList& remote, const std::set<Id>& dead,
                      std::vector<std::string>* status_changes) {
  if (local.empty()) return false;  // not in a group (never joined, or left)
  bool changed = false;
  for (const auto& kv : remote) {
    if (dead.count(kv.first)) continue;
    auto it = local.find(kv.first);
    if (it == local.end()) {
      local.emplace(kv.first, kv.second);
      changed = true;
      continue;
    }
    Membership& m = it->second;
    const Membership& rm = kv.second;
    if (m.last_active < rm.last_active || (m.last_active == rm.last_active && rm.status == Status::Failed &&
                                           m.status != Status::Failed)) {
      if (m.status != rm.status && status_changes)
        status_changes->push_back("Updating membership for " + kv.first.address + ": " + status_name(m.status) +
                                  " -> " + status_name(rm.status));
      m = rm;
      changed = true;
    }
  }
  return changed;
}

static std::string list_table(const MembershipList& l, bool active_only) {
  std::vector<std::vector<std::string>> rows;
  for (const auto& kv : l) {
    if (active_only && kv.second.status != Status::Active) continue;
    rows.push_back({kv.first.address, format_time_us(kv.first.timestamp), status_name(kv.second.status),
                    format_time_us(kv.second.last_active)});
  }
  return make_table({"address", "timestamp", "status", "last_active"}, rows);
}

MembershipService::MembershipService(MembershipConfig cfg) : cfg_(std::move(cfg)) {
  id_.address = cfg_.host + ":" + std::to_string(cfg_.port);
  id_.timestamp = own_us();
}

MembershipService::~MembershipService() { stop(); }

void MembershipService::start() {
  sock_ = udp_bind(cfg_.bind_host, cfg_.port);
  out_line("Address is " + id_.address);
  rx_ = std::thread([this] { receiver_loop(); });
  ping_ = std::thread([this] { pinger_loop(); });
  det_ = std::thread([this] { detector_loop(); });
}

void MembershipService::stop() {
  if (stop_.exchange(true)) return;
  if (rx_.joinable()) rx_.join();
  if (ping_.joinable()) ping_.join();
  if (det_.joinable()) det_.join();
  sock_.reset();
}

Id MembershipService::id() const {
  std::lock_guard<std::mutex> g(mu_);
  return id_;
}

MembershipList MembershipService::snapshot() const {
  std::lock_guard<std::mutex> g(mu_);
  return list_;
}

std::set<Id> MembershipService::active_ids() const {
  std::lock_guard<std::mutex> g(mu_);
  std::set<Id> s;
  for (const auto& kv : list_)
    if (kv.second.status == Status::Active) s.insert(kv.first);
  return s;
}

std::vector<Id> MembershipService::active_sorted() const {
  auto s = active_ids();
  return std::vector<Id>(s.begin(), s.end());
}

std::vector<Id> MembershipService::neighbors() const {
  std::lock_guard<std::mutex> g(mu_);
  return symmetric_ring_neighbors(list_, id_, cfg_.k,
                                  [](const std::pair<const Id, Membership>& e) { return e.second.status == Status::Active; });
}

void MembershipService::partition(const std::string& addr) {
  std::lock_guard<std::mutex> g(part_mu_);
  partitioned_.insert(addr);
}

void MembershipService::heal() {
  std::lock_guard<std::mutex> g(part_mu_);
  partitioned_.clear();
}

bool MembershipService::blocked(const std::string& addr) {
  if (paused_.load()) return true;
  {
    std::lock_guard<std::mutex> g(part_mu_);
    if (partitioned_.count(addr)) return true;
  }
  const double p = drop_rate_.load();
  if (p > 0) {
    std::lock_guard<std::mutex> g(rng_mu_);
    return std::uniform_real_distribution<double>(0, 1)(rng_) < p;
  }
  return false;
}

void MembershipService::send(const std::string& addr, const Message& m) {
  if (blocked(addr)) return;
  try {
    if (!udp_send(sock_.get(), resolve_addr(addr), encode_message(m)))
      DMLC_LOG_WARN("Error sending message to " << addr);
    else
      sent_++;
  } catch (const std::exception& e) {
    DMLC_LOG_WARN("Error sending message to " << addr << ": " << e.what());
  }
}

void MembershipService::join(const std::string& introducer) {
  Message m;
  m.type = MsgType::Join;
  {
    std::lock_guard<std::mutex> g(mu_);
    id_.timestamp = own_us();  // new incarnation
    m.sender = id_;
  }
  send(introducer, m);
}

void MembershipService::leave() {
  std::vector<Id> nbrs = neighbors();
  Message m;
  m.type = MsgType::Leave;
  {
    std::lock_guard<std::mutex> g(mu_);
    m.sender = id_;
    m.last_active = own_us();
    const std::string msg = "Leaving group...\nLast membership list:\n" + list_table(list_, false);
    DMLC_LOG_INFO(msg);
    out_line(msg);
  }
  for (const auto& n : nbrs) send(n.address, m);
  std::lock_guard<std::mutex> g(mu_);
  list_.clear();
  last_neighbors_.clear();
}

void MembershipService::receiver_loop() {
  std::vector<char> buf(65536);
  while (!stop_.load()) {
    sockaddr_in from{};
    int n = udp_recv(sock_.get(), buf.data(), buf.size(), 200, &from);
    if (n <= 0) continue;
    Message m;
    try {
      m = decode_message(buf.data(), (size_t)n);
    } catch (const std::exception&) {
      continue;  // malformed datagram
    }
    if (blocked(m.sender.address)) continue;
    received_++;
    std::vector<std::string> changes;
    switch (m.type) {
      case MsgType::Ping: {
        bool in_group;
        Id self;
        {
          std::lock_guard<std::mutex> g(mu_);
          merge_membership(list_, m.list, dead_, &changes);
          in_group = !list_.empty();
          self = id_;
        }
        if (in_group) {
          Message ack;
          ack.type = MsgType::Ack;
          ack.sender = self;
          ack.last_active = own_us();
          send(m.sender.address, ack);
        }
        break;
      }
      case MsgType::Ack: {
        std::lock_guard<std::mutex> g(mu_);
        MembershipList one;
        one[m.sender] = Membership{Status::Active, m.last_active};
        merge_membership(list_, one, dead_, &changes);
        break;
      }
      case MsgType::Join: {
        Message w;
        w.type = MsgType::Welcome;
        {
          std::lock_guard<std::mutex> g(mu_);
          for (auto& kv : list_)  // fail older incarnations of the same address (fast rejoin)
            if (kv.first.address == m.sender.address && kv.first != m.sender) kv.second.status = Status::Failed;
          dead_.erase(m.sender);
          list_[m.sender] = Membership{Status::Active, m.sender.timestamp};
          auto it = list_.find(id_);
          if (it != list_.end()) it->second = Membership{Status::Active, own_us()};
          w.sender = id_;
          w.list = list_;
        }
        DMLC_LOG_INFO("Join from " << m.sender.address);
        send(m.sender.address, w);
        break;
      }
      case MsgType::Welcome: {
        std::string msg;
        {
          std::lock_guard<std::mutex> g(mu_);
          list_ = m.list;
          for (const auto& d : dead_) list_.erase(d);
          msg = "Joined!\nInitial membership list:\n" + list_table(list_, false);
        }
        DMLC_LOG_INFO(msg);
        out_line(msg);
        break;
      }
      case MsgType::Leave: {
        std::lock_guard<std::mutex> g(mu_);
        auto it = list_.find(m.sender);
        if (it != list_.end() && it->second.status == Status::Active) {
          it->second.status = Status::Failed;
          it->second.last_active = std::max(it->second.last_active, m.last_active);
          changes.push_back("Updating membership for " + m.sender.address + ": Active -> Failed (left)");
        }
        break;
      }
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      note_heard_locked();
    }
    for (const auto& c : changes) {
      DMLC_LOG_INFO(c);
      out_line(c);
    }
  }
}

void MembershipService::note_heard_locked() {
  const int64_t st = steady_us();
  for (const auto& kv : list_) {
    auto& h = heard_[kv.first];
    if (h.second == 0 || kv.second.last_active > h.first) h = {kv.second.last_active, st};
  }
  for (auto it = heard_.begin(); it != heard_.end();) it = list_.count(it->first) ? std::next(it) : heard_.erase(it);
}

void MembershipService::pinger_loop() {
  std::vector<Id> active_neighbors;
  while (!stop_.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.ping_ms));
    if (paused_.load()) continue;
    Message m;
    m.type = MsgType::Ping;
    std::vector<Id> nbrs;
    {
      std::lock_guard<std::mutex> g(mu_);
      const int64_t now = own_us();
      auto it = list_.find(id_);
      if (it != list_.end()) it->second = Membership{Status::Active, now};
      // tombstone GC, aged by the local time since the entry last advanced
      note_heard_locked();
      const int64_t st = steady_us();
      for (auto jt = list_.begin(); jt != list_.end();) {
        if (jt->second.status == Status::Failed && st - heard_[jt->first].second > (int64_t)cfg_.tombstone_ms * 1000) {
          dead_.insert(jt->first);
          heard_.erase(jt->first);
          jt = list_.erase(jt);
        } else {
          ++jt;
        }
      }
      m.sender = id_;
      m.list = list_;
      nbrs = symmetric_ring_neighbors(list_, id_, cfg_.k, [](const std::pair<const Id, Membership>& e) {
        return e.second.status == Status::Active;
      });
    }
    if (nbrs != active_neighbors) {
      std::string s;
      for (const auto& n : nbrs) s += " " + n.address;
      DMLC_LOG_INFO("Active neighbors have changed:" << s);
      active_neighbors = nbrs;
    }
    for (const auto& n : active_neighbors) send(n.address, m);
  }
}

void MembershipService::detector_loop() {
  while (!stop_.load()) {
    std::vector<std::string> msgs;
    {
      std::lock_guard<std::mutex> g(mu_);
      note_heard_locked();
      const int64_t now = steady_us();
      if (!paused_.load()) {
        for (const auto& n : last_neighbors_) {
          auto it = list_.find(n);
          if (it == list_.end() || it->second.status != Status::Active) continue;
          const int64_t el = now - heard_[n].second;
          if (el > (int64_t)cfg_.fail_ms * 1000) {
            it->second.status = Status::Failed;
            msgs.push_back("Detected failure of " + n.debug() + " that hasn't been updated for " +
                           std::to_string(el / 1000) + " ms");
          }
        }
      }
      last_neighbors_ = symmetric_ring_neighbors(list_, id_, cfg_.k, [](const std::pair<const Id, Membership>& e) {
        return e.second.status == Status::Active;
      });
    }
    for (const auto& s : msgs) {
      DMLC_LOG_WARN(s);
      out_line(s);
    }
    for (int slept = 0; slept < cfg_.detect_ms && !stop_.load(); slept += 50)
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

}  // namespace ctl
}  // namespace dmlc
