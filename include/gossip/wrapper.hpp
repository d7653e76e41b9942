// wrapper.hpp -- drop-in Peer facade (reference: wrapper.hpp:7-19, wrapper.cpp:3-35).
// Peer(configFile) parses network.txt with NetworkConfig and owns the
// simulated network it describes; start() runs it (blocking, like the
// reference's accept loop) until every message has spread or stop() is
// called from another thread / a signal handler.
#pragma once

#include <memory>
#include <string>

#include "gossip/config.hpp"
#include "gossip/network.hpp"
#include "gossip/peer.hpp"

class Peer {
public:
    Peer(const std::string& configFile);
    ~Peer();

    void start();
    void stop();
    bool isRunning() const;

    // -- extension -----------------------------------------------------------
    std::shared_ptr<GossipNetwork> network() const { return net_; }
    const NetworkConfig& config() const { return config_; }

private:
    std::unique_ptr<PeerNode> node;
    NetworkConfig config_;
    std::shared_ptr<GossipNetwork> net_;
};
