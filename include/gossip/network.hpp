// network.hpp -- GossipNetwork: the reference's seed/peer deployment as one
// deterministic, engine-backed simulation (libgossip_hip, include/gossip/gossip.h).
//
// One round = one second of the reference's clock.  Per round the engine runs
// churn -> liveness pings (pingLoop, peer.cpp:320-355) -> message generation
// (messageGenerationLoop, peer.cpp:357-379) -> push + Message-List dedup
// (broadcastMessage/handleClient, peer.cpp:255-318).  For small networks
// (<= kTraceMax peers) the run is traced so that the reference's per-peer
// and per-seed log files, message lists and sentTo sets can be reproduced.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "gossip/config.hpp"
#include "gossip/gossip.h"
#include "gossip/info.hpp"
#include "gossip/peer.hpp"
#include "gossip/seed.hpp"

struct SimOptions {
    uint64_t n_peers = 8;
    uint32_t rng_seed = 0x5EED0001u;
    std::string graph = "ref_bootstrap";  // or "powerlaw"
    uint32_t list_len = 6;
    uint32_t origins = 0;                 // 0: every peer generates (reference); k: k Philox-chosen origins
    uint32_t messages_per_origin = 10;    // max_messages (config.cpp:36, peer.cpp:358)
    uint32_t message_every = 5;           // message_interval in rounds (peer.cpp:377)
    uint32_t ping_every = 15;             // 5 s tick gated by ping_interval 13 s (peer.cpp:329-330,353)
    uint32_t max_missed = 3;              // max_missed_pings (peer.cpp:337)
    uint32_t churn_threshold = 0;         // peer dies in round r iff philox < threshold
    uint32_t max_rounds = 4096;
    uint32_t min_rounds = 0;
    std::vector<std::pair<uint32_t, uint32_t>> kills;  // (peer, round): "Ctrl+C" (README.md:6)
    int device = -1;
    // vertex partitions (gossip_group_*: one per GPU 0..n_gpus-1, RCCL collectives inside the library;
    // when fewer GPUs are visible, every part on `device` with device-copy exchange).  Traced
    // networks (<= kTraceMax peers) keep one partition: their per-peer views read the whole overlay.
    uint32_t n_gpus = 1;
    std::string log_dir;                  // reference-format logs (small networks)
    std::vector<std::pair<std::string, int>> addresses;  // optional ip:port per peer (default: peer_address())

    // Reference keys (ping_interval, message_interval, max_messages,
    // max_missed_pings) plus simulation keys: n_peers, rng_seed, graph,
    // list_len, origins, churn_ppm, max_rounds, min_rounds, kills=p@r,...,
    // device, n_gpus, log_dir.
    static SimOptions fromConfig(const NetworkConfig& cfg);
};

class GossipNetwork : public std::enable_shared_from_this<GossipNetwork> {
public:
    static constexpr uint64_t kTraceMax = 4096;

    GossipNetwork(std::vector<PeerInfo> seeds, SimOptions opt);
    GossipNetwork(const NetworkConfig& cfg, SimOptions opt);
    ~GossipNetwork();
    GossipNetwork(const GossipNetwork&) = delete;
    GossipNetwork& operator=(const GossipNetwork&) = delete;

    bool start();   // bootstrap: overlay, seed registrations, schedule (false + std::cerr on failure)
    int step();     // one round; 1 when finished, 0 if not, < 0 on error
    bool run();     // rounds until finished or stop()
    void stop() { stop_ = true; }
    bool isRunning() const { return started_ && !finished_ && !stop_; }
    bool finished() const { return finished_; }

    uint64_t size() const { return opt_.n_peers; }
    uint32_t messages() const { return M_; }
    const SimOptions& options() const { return opt_; }
    PeerInfo peerInfo(uint64_t id) const;
    long long idOf(const std::string& ip, int port) const;
    Message message(uint32_t m) const;
    const std::vector<gossip_round_stats>& rounds() const { return rounds_; }
    std::vector<gossip_dead_report> reports() const;
    std::vector<SeedNode*> seeds();
    std::shared_ptr<PeerNode> peer(uint64_t id);
    gossip_ctx* ctx() const { return ctx_; }        // single partition (null when partitioned)
    gossip_group* group() const { return group_; }  // partitioned (n_gpus > 1)

    // traced views (size() <= kTraceMax)
    bool traced() const { return trace_; }
    std::vector<uint32_t> rowOf(uint64_t id) const;             // out-neighbours (CSR row, bootstrap)
    bool edgeLive(uint64_t id, uint32_t to) const;              // not dropped by liveness
    long receiptRound(uint64_t id, uint32_t m) const;           // -1: never received / generated
    std::vector<uint32_t> sentTo(uint64_t id, uint32_t m) const;

    void writeLogs(const std::string& dir) const;

private:
    std::vector<PeerInfo> seedInfo_;
    SimOptions opt_;
    uint32_t M_ = 0, W_ = 0;
    gossip_ctx* ctx_ = nullptr;
    uint64_t groupReportCount() const;  // ~0: a part's count is unreadable (report buffer overflow)
    uint64_t mergedReports_ = 0;        // reports behind the seed removals merged so far (partitioned runs)
    gossip_group* group_ = nullptr;
    bool started_ = false, finished_ = false, trace_ = false;
    std::atomic<bool> stop_{false};
    std::vector<uint32_t> origin_, injectRound_;
    std::vector<gossip_round_stats> rounds_;
    std::vector<std::unique_ptr<SeedNode>> seedNodes_;
    // trace state
    std::vector<uint64_t> rp_;
    std::vector<uint32_t> col_;
    std::vector<uint64_t> seen_;               // n * W, current
    std::vector<int32_t> recvRound_;           // n * M: round of first receipt (-1 none)
    std::vector<uint8_t> alive_;               // current
    std::vector<std::vector<uint8_t>> aliveAt_;  // per round (after churn/kills)
    std::vector<int32_t> maskRound_;           // per edge: round masked (-1 live)
    std::vector<int32_t> deathRound_;          // per peer

    void captureRound(uint32_t r);
    void seedRemovalsFromReports();  // partitioned runs: each round's removals from the merged reports
};
