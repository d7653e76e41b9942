// gossip_network.cpp -- GossipNetwork: seed bootstrap, rounds and traces on
// top of the libgossip_hip C-ABI (the only compute path; no CPU fallback).
#include <algorithm>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>

#include "gossip/formats.hpp"
#include "gossip/network.hpp"

namespace {

uint32_t churn_threshold_from_ppm(long long ppm) {
    if (ppm <= 0) return 0;
    const long double t = (long double)ppm * 4294967296.0L / 1000000.0L;
    return (uint32_t)std::min<long double>(t + 0.5L, 4294967295.0L);
}

std::vector<std::pair<uint32_t, uint32_t>> parse_kills(const std::string& s) {
    std::vector<std::pair<uint32_t, uint32_t>> out;
    std::stringstream ss(s);
    std::string item;
    while (std::getline(ss, item, ',')) {
        const size_t at = item.find('@');
        if (at == std::string::npos) continue;
        out.emplace_back((uint32_t)std::stoul(item.substr(0, at)), (uint32_t)std::stoul(item.substr(at + 1)));
    }
    return out;
}

}  // namespace

SimOptions SimOptions::fromConfig(const NetworkConfig& c) {
    SimOptions o;
    o.messages_per_origin = (uint32_t)c.getMaxMessages();
    o.message_every = (uint32_t)c.getMessageInterval();
    o.ping_every = (uint32_t)((c.getPingInterval() + 4) / 5 * 5);  // 5 s tick gated by ping_interval
    o.max_missed = (uint32_t)c.getMaxMissedPings();
    o.n_peers = (uint64_t)c.getInt("n_peers", 8);
    o.rng_seed = (uint32_t)c.getInt("rng_seed", 0x5EED0001);
    o.graph = c.getString("graph", o.n_peers <= 4096 ? "ref_bootstrap" : "powerlaw");
    o.list_len = (uint32_t)c.getInt("list_len", 6);
    o.origins = (uint32_t)c.getInt("origins", 0);
    o.churn_threshold = churn_threshold_from_ppm(c.getInt("churn_ppm", 0));
    o.max_rounds = (uint32_t)c.getInt("max_rounds", 4096);
    o.min_rounds = (uint32_t)c.getInt("min_rounds", 0);
    o.kills = parse_kills(c.getString("kills", ""));
    o.device = (int)c.getInt("device", -1);
    o.n_gpus = (uint32_t)std::max<long long>(1, c.getInt("n_gpus", 1));
    o.log_dir = c.getString("log_dir", "");
    return o;
}

GossipNetwork::GossipNetwork(std::vector<PeerInfo> seeds, SimOptions opt) : seedInfo_(std::move(seeds)), opt_(std::move(opt)) {}

GossipNetwork::GossipNetwork(const NetworkConfig& cfg, SimOptions opt) : opt_(std::move(opt)) {
    for (const auto& s : cfg.getSeedNodes()) seedInfo_.push_back(PeerInfo{s.ip, s.port, {}});
}

GossipNetwork::~GossipNetwork() {
    if (ctx_) gossip_destroy(ctx_);
    if (group_) gossip_group_destroy(group_);
}

PeerInfo GossipNetwork::peerInfo(uint64_t id) const {
    if (id < opt_.addresses.size()) return PeerInfo{opt_.addresses[id].first, opt_.addresses[id].second, {}};
    const gossip::PeerAddress a = gossip::peer_address(id, opt_.n_peers);
    return PeerInfo{a.ip, a.port, {}};
}

long long GossipNetwork::idOf(const std::string& ip, int port) const {
    for (uint64_t i = 0; i < opt_.n_peers && i < kTraceMax; ++i) {
        const PeerInfo p = peerInfo(i);
        if (p.ip == ip && p.port == port) return (long long)i;
    }
    return -1;
}

Message GossipNetwork::message(uint32_t m) const {
    const PeerInfo o = peerInfo(origin_.at(m));
    Message msg;
    msg.content = gossip::message_content({o.ip, o.port});
    msg.timestamp = gossip::message_timestamp(injectRound_.at(m));
    msg.sourceIP = o.ip;
    msg.sourcePort = o.port;
    msg.msgNumber = (int)(m % opt_.messages_per_origin);
    msg.hash = gossip::message_hash(msg.content, msg.timestamp, msg.sourceIP);  // peer.cpp:135-159
    return msg;
}

bool GossipNetwork::start() {
    if (started_) return true;
    const uint64_t n = opt_.n_peers;
    const uint64_t n_origins = opt_.origins ? opt_.origins : n;
    const uint64_t M = n_origins * opt_.messages_per_origin;
    if (n == 0 || M == 0 || M > 512) {
        std::cerr << "Error creating gossip network: " << M
                  << " concurrent messages (set origins= so that origins * max_messages <= 512)" << std::endl;
        return false;
    }
    M_ = (uint32_t)M;
    W_ = (M_ + 63) / 64;
    gossip_config cfg{};
    cfg.n_peers = n;
    cfg.n_msgs = M_;
    cfg.rng_seed = opt_.rng_seed;
    cfg.graph_model = opt_.graph == "powerlaw" ? GOSSIP_GRAPH_POWERLAW : GOSSIP_GRAPH_REF_BOOTSTRAP;
    cfg.list_len = opt_.list_len;
    cfg.n_seeds = (uint32_t)std::max<size_t>(seedInfo_.size(), 1);
    cfg.churn_threshold = opt_.churn_threshold;
    cfg.ping_every = opt_.ping_every;
    cfg.max_missed = opt_.max_missed;
    cfg.max_rounds = opt_.max_rounds;
    cfg.min_rounds = opt_.min_rounds;
    cfg.device = opt_.device;
    trace_ = n <= kTraceMax;
    const uint32_t parts = trace_ ? 1u : std::max<uint32_t>(1, opt_.n_gpus);
    gossip_status st = GOSSIP_OK;
    if (parts > 1) {
        // parts on GPUs device, device+1, ...; with fewer GPUs visible than that, every part on
        // `device`, exchanging by device copies (the single-GPU rehearsal of the partitioned path).
        // Any other failure (RCCL, memory) is reported, not papered over.
        int32_t ndev = 0;
        st = gossip_device_count(&ndev);
        const int32_t base = std::max(opt_.device, 0);
        const bool distinct = (int64_t)ndev >= (int64_t)base + parts;
        std::vector<int32_t> devs(parts);
        for (uint32_t p = 0; p < parts; ++p) devs[p] = distinct ? base + (int32_t)p : base;
        if (st == GOSSIP_OK) st = gossip_group_create(&cfg, parts, devs.data(), &group_);
        if (st == GOSSIP_OK) st = gossip_group_build_graph(group_);
    } else {
        st = gossip_create(&cfg, &ctx_);
        if (st == GOSSIP_OK) st = gossip_build_graph(ctx_);
    }
    // messageGenerationLoop (peer.cpp:357-379): origin o's k-th message at round k * message_every
    std::vector<uint32_t> origins(n_origins);
    if (st == GOSSIP_OK) {
        if (opt_.origins) st = gossip_pick_origins(n, opt_.rng_seed, (uint32_t)n_origins, origins.data());
        else
            for (uint64_t i = 0; i < n; ++i) origins[i] = (uint32_t)i;
    }
    origin_.resize(M_);
    injectRound_.resize(M_);
    for (uint64_t oi = 0; oi < n_origins; ++oi)
        for (uint32_t k = 0; k < opt_.messages_per_origin; ++k) {
            origin_[oi * opt_.messages_per_origin + k] = origins[oi];
            injectRound_[oi * opt_.messages_per_origin + k] = k * opt_.message_every;
        }
    if (st == GOSSIP_OK)
        st = group_ ? gossip_group_inject(group_, origin_.data(), injectRound_.data(), M_)
                    : gossip_inject(ctx_, origin_.data(), injectRound_.data(), M_);
    if (st == GOSSIP_OK && !opt_.kills.empty()) {
        std::vector<uint32_t> kp, kr;
        for (const auto& k : opt_.kills) {
            kp.push_back(k.first);
            kr.push_back(k.second);
        }
        st = group_ ? gossip_group_schedule_kills(group_, kp.data(), kr.data(), (uint32_t)kp.size())
                    : gossip_schedule_kills(ctx_, kp.data(), kr.data(), (uint32_t)kp.size());
    }
    if (st == GOSSIP_OK) st = group_ ? gossip_group_reset(group_) : gossip_reset(ctx_);
    if (st != GOSSIP_OK) {
        std::cerr << "Error starting gossip network: " << gossip_strerror(st) << ": " << gossip_last_error() << std::endl;
        return false;
    }
    // seeds (seed.cpp:15-90) and the bootstrap registrations (peer.cpp:63-72 -> seed.cpp:109-129)
    for (const PeerInfo& s : seedInfo_) {
        seedNodes_.emplace_back(new SeedNode(s.ip, s.port));
        seedNodes_.back()->setLogDir(opt_.log_dir);
        seedNodes_.back()->setClock(gossip::kEpochSeconds);
        seedNodes_.back()->start();
    }
    if (trace_) {
        const size_t q = std::min(seedNodes_.size(), seedNodes_.size() / 2 + 1);
        for (uint64_t i = 0; i < n; ++i) {
            const PeerInfo p = peerInfo(i);
            for (size_t s = 0; s < q; ++s) {
                seedNodes_[s]->log("New client connection accepted");
                seedNodes_[s]->handleRequest(gossip::register_json(p.ip, p.port));
            }
        }
        uint32_t words = 0, xw = 0;
        uint64_t nl = 0, ne = 0;
        gossip_get_shape(ctx_, &words, &xw, &nl, &ne);
        rp_.resize(n + 1);
        col_.resize(std::max<uint64_t>(ne, 1));
        gossip_read_csr(ctx_, rp_.data(), col_.data());
        col_.resize(ne);
        seen_.assign(n * W_, 0);
        recvRound_.assign(n * M_, -1);
        alive_.assign(n, 1);
        maskRound_.assign(ne, -1);
        deathRound_.assign(n, -1);
    }
    started_ = true;
    return true;
}

void GossipNetwork::captureRound(uint32_t r) {
    const uint64_t n = opt_.n_peers;
    std::vector<uint8_t> alive(n);
    gossip_read_alive(ctx_, alive.data());
    for (uint64_t v = 0; v < n; ++v)
        if (alive_[v] && !alive[v]) deathRound_[v] = (int32_t)r;
    alive_ = alive;
    aliveAt_.push_back(alive);
    std::vector<uint64_t> seen(n * W_);
    gossip_read_seen(ctx_, seen.data());
    for (uint64_t i = 0; i < n * W_; ++i) {
        for (uint64_t x = seen[i] & ~seen_[i]; x; x &= x - 1) {
            const uint32_t m = (uint32_t)((i % W_) * 64 + __builtin_ctzll(x));
            recvRound_[(i / W_) * M_ + m] = (int32_t)r;
        }
    }
    seen_.swap(seen);
    std::vector<uint64_t> rp(n + 1);
    std::vector<uint32_t> col(std::max<size_t>(col_.size(), 1));
    gossip_read_csr(ctx_, rp.data(), col.data());
    for (size_t e = 0; e < col_.size(); ++e)
        if ((col[e] & 0x80000000u) && maskRound_[e] < 0) maskRound_[e] = (int32_t)r;
    // dead-node reports of this round go to the seeds the reporter registered with
    const size_t q = std::min(seedNodes_.size(), seedNodes_.size() / 2 + 1);
    for (const gossip_dead_report& rep : reports()) {
        if (rep.round != r) continue;
        const PeerInfo d = peerInfo(rep.dead);
        for (size_t s = 0; s < q; ++s) {
            seedNodes_[s]->setClock(gossip::kEpochSeconds + r);
            seedNodes_[s]->log("New client connection accepted");
            seedNodes_[s]->handleRequest(gossip::dead_node_json(d.ip, d.port));
        }
    }
}

int GossipNetwork::step() {
    if (!started_ && !start()) return GOSSIP_ESTATE;
    if (finished_) return 1;
    gossip_round_stats st{};
    const int rc = group_ ? gossip_group_step(group_, &st) : gossip_step(ctx_, &st);
    if (rc < 0) {
        std::cerr << "Error in gossip round: " << gossip_strerror(rc) << ": " << gossip_last_error() << std::endl;
        return rc;
    }
    rounds_.push_back(st);
    if (trace_) captureRound(st.round);
    if (rc == 1) finished_ = true;
    // a partitioned run's seed removals come from the merged reports (single-partition stats carry them every
    // round): after a round that added reports while they are few (or traced), else once the run ends.  A
    // round without new reports has no removals (its stats carry 0), so nothing is merged again for it.
    if (group_) {
        const uint64_t cnt = finished_ || trace_ ? ~0ull : groupReportCount();
        if (finished_ || trace_ || (cnt < (1u << 20) && cnt != mergedReports_)) {
            seedRemovalsFromReports();
            mergedReports_ = cnt;
        }
    }
    return rc;
}

bool GossipNetwork::run() {
    if (!started_ && !start()) return false;
    while (!finished_ && !stop_) {
        if (step() < 0) return false;
    }
    if (finished_ && !opt_.log_dir.empty() && trace_) writeLogs(opt_.log_dir);
    return true;
}

std::vector<gossip_dead_report> GossipNetwork::reports() const {
    uint64_t count = 0;
    if (group_) {
        if (gossip_group_read_reports(group_, nullptr, 0, &count) != GOSSIP_OK || count == 0) return {};
        std::vector<gossip_dead_report> out(count);
        gossip_group_read_reports(group_, out.data(), count, &count);
        return out;
    }
    if (!ctx_ || gossip_read_reports(ctx_, nullptr, 0, &count) != GOSSIP_OK || count == 0) return {};
    std::vector<gossip_dead_report> out(count);
    gossip_read_reports(ctx_, out.data(), count, &count);
    return out;
}

// Reports held by the parts of a group (their counters only: no merge); a part whose count cannot be read
// (its report buffer overflowed: GOSSIP_EOVERFLOW) makes the total "many" (~0), so the merge waits for the
// end of the run instead of dropping that part's reports
uint64_t GossipNetwork::groupReportCount() const {
    uint64_t total = 0;
    gossip_ctx* part = nullptr;
    for (uint32_t p = 0; group_ && gossip_group_part(group_, p, &part) == GOSSIP_OK; ++p) {
        uint64_t n = 0;
        if (gossip_read_reports(part, nullptr, 0, &n) != GOSSIP_OK) return ~0ull;
        total += n;
    }
    return total;
}

// The registry drops a peer on its first report (SeedNode::handleDeadNode,
// seed.cpp:158-167): a partitioned run's per-round stats get their seed
// removals from the merged report list.
void GossipNetwork::seedRemovalsFromReports() {
    std::map<uint32_t, uint32_t> first;  // dead peer -> round of its first report
    for (const gossip_dead_report& r : reports()) {
        auto it = first.find(r.dead);
        if (it == first.end() || r.round < it->second) first[r.dead] = r.round;
    }
    for (gossip_round_stats& st : rounds_) st.seed_removals = 0;
    for (const auto& kv : first)
        for (gossip_round_stats& st : rounds_)
            if (st.round == kv.second) {
                st.seed_removals++;
                break;
            }
}

std::vector<SeedNode*> GossipNetwork::seeds() {
    std::vector<SeedNode*> out;
    for (auto& s : seedNodes_) out.push_back(s.get());
    return out;
}

std::shared_ptr<PeerNode> GossipNetwork::peer(uint64_t id) {
    return std::make_shared<PeerNode>(shared_from_this(), (unsigned)id);
}

std::vector<uint32_t> GossipNetwork::rowOf(uint64_t id) const {
    if (!trace_) return {};
    std::vector<uint32_t> out;
    for (uint64_t e = rp_[id]; e < rp_[id + 1]; ++e) out.push_back(col_[e] & 0x7FFFFFFFu);
    return out;
}

bool GossipNetwork::edgeLive(uint64_t id, uint32_t to) const {
    if (!trace_) return false;
    for (uint64_t e = rp_[id]; e < rp_[id + 1]; ++e)
        if ((col_[e] & 0x7FFFFFFFu) == to) return maskRound_[e] < 0;
    return false;
}

long GossipNetwork::receiptRound(uint64_t id, uint32_t m) const {
    return trace_ ? (long)recvRound_[id * M_ + m] : -1;
}

// broadcastMessage's sentTo (peer.cpp:310-316): the live out-neighbours that
// were alive in the round this peer pushed m (its generation round, or the
// round after it first received m).
std::vector<uint32_t> GossipNetwork::sentTo(uint64_t id, uint32_t m) const {
    std::vector<uint32_t> out;
    const long got = receiptRound(id, m);
    if (got < 0) return out;
    const long push = origin_[m] == id && (long)injectRound_[m] == got ? got : got + 1;
    if (push >= (long)aliveAt_.size() || !aliveAt_[push][id]) return out;
    for (uint64_t e = rp_[id]; e < rp_[id + 1]; ++e) {
        const uint32_t c = col_[e] & 0x7FFFFFFFu;
        if ((maskRound_[e] < 0 || maskRound_[e] > push) && aliveAt_[push][c]) out.push_back(c);
    }
    return out;
}

void GossipNetwork::writeLogs(const std::string& dir) const {
    if (!trace_ || opt_.n_peers > 60000) return;
    std::vector<Message> msgs;
    for (uint32_t m = 0; m < M_; ++m) msgs.push_back(message(m));
    for (uint64_t v = 0; v < opt_.n_peers; ++v) {
        const PeerInfo me = peerInfo(v);
        std::ofstream f(dir + "/peer_" + std::to_string(me.port) + "_output.txt", std::ios::app);
        const std::time_t t0 = (std::time_t)gossip::kEpochSeconds;
        f << gossip::peer_log_line(t0, "Peer node started on port " + std::to_string(me.port));  // peer.cpp:61
        for (uint32_t c : rowOf(v)) {                                                              // peer.cpp:248
            const PeerInfo p = peerInfo(c);
            f << gossip::peer_log_line(t0, "Connected to peer: " + p.ip + ":" + std::to_string(p.port));
        }
        std::map<long, std::vector<std::string>> events;
        for (uint64_t e = rp_[v]; e < rp_[v + 1]; ++e) {
            if (maskRound_[e] < 0) continue;  // peer.cpp:389
            const PeerInfo p = peerInfo(col_[e] & 0x7FFFFFFFu);
            events[maskRound_[e]].push_back("Peer disconnected: " + p.ip + ":" + std::to_string(p.port));
        }
        for (uint32_t m = 0; m < M_; ++m) {
            const long r = receiptRound(v, m);
            if (r < 0) continue;
            const bool own = origin_[m] == v && (long)injectRound_[m] == r;
            events[r].push_back((own ? "Generated message: " : "Received new message: ") + msgs[m].content);
        }
        for (const auto& kv : events)
            for (const std::string& s : kv.second) f << gossip::peer_log_line(t0 + kv.first, s);
    }
}
