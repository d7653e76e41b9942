// seed.hpp -- drop-in SeedNode (reference: seed.hpp:9-34, seed.cpp:15-204).
//
// A seed is the peer registry: addPeer() registers (seed.cpp:153-156),
// getPeerList() returns every registered peer (seed.cpp:169-178),
// handleDeadNode() erases a reported peer and logs "Removed dead peer" on
// the first removal (seed.cpp:158-167).  There is no socket server: the
// registration and dead_node messages arrive from the simulated peers of a
// GossipNetwork (or from the caller), and every message the reference would
// have logged is appended to seed_<port>_output.txt when logging is enabled.
#pragma once

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gossip/info.hpp"

class SeedNode {
public:
    SeedNode(const std::string& ip, int port);
    ~SeedNode();

    bool start();  // marks the seed running; logs "Seed node started on port <p>" (seed.cpp:59)
    void stop();

    void addPeer(const PeerInfo& peer);
    void handleDeadNode(const std::string& deadIP, int deadPort);
    std::vector<PeerInfo> getPeerList();

    // -- extension --------------------------------------------------------------
    const std::string& ip() const { return ip_; }
    int port() const { return port_; }
    bool isRunning() const { return running_; }
    // Handle one request in the reference wire format ({"type":"register",...}
    // or {"type":"dead_node",...}); returns the response a reference seed
    // would send ("" for dead_node), logging as seed.cpp:92-151 does.
    std::string handleRequest(const std::string& json);
    // Logging: enabled with a directory; timestamps come from the simulation clock.
    void setLogDir(const std::string& dir);
    void setClock(long long unix_seconds) { clock_ = unix_seconds; }
    void log(const std::string& message);
    size_t size();

private:
    std::string ip_;
    int port_;
    std::atomic<bool> running_{false};  // stop() may come from another thread (main.cpp:14-22)
    std::unordered_map<PeerInfo, std::chrono::system_clock::time_point, PeerInfoHash> peers_;
    std::vector<PeerInfo> order_;  // registration order (a deterministic peer_list)
    std::mutex mu_;
    std::string logPath_;
    std::atomic<long long> clock_{0};  // simulation clock of the log stamps (set while peers register)
};
