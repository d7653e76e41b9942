// peer.hpp -- drop-in PeerNode and the reference's message types
// (reference: peer.hpp:14-81).
//
// In the reference every PeerNode is a process with sockets and threads.
// Here a PeerNode is a handle to one peer of a GossipNetwork, the
// engine-backed simulation of the whole overlay; its public surface
// (constructor, start, stop, isRunning) is the reference's, plus read-only
// views of the state the reference keeps privately (connectedPeers,
// messageList with sentTo).
#pragma once

#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <queue>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "gossip/info.hpp"
#include "gossip/seed.hpp"  // the reference's peer.hpp pulls PeerInfo in through seed.hpp

struct Message {
    std::string content;
    std::string timestamp;
    std::string sourceIP;
    int sourcePort;
    int msgNumber;
    std::string hash;
};

struct MessageTracker {
    Message msg;
    std::set<std::pair<std::string, int>> sentTo;
};

struct PairHash {
    template <class T1, class T2>
    std::size_t operator()(const std::pair<T1, T2>& p) const {
        return std::hash<T1>()(p.first) ^ (std::hash<T2>()(p.second) << 1);
    }
};

class GossipNetwork;

class PeerNode {
public:
    // Reference constructor: a peer that bootstraps from `seeds`.  Started on
    // its own it is the first arrival of an empty network (F8: it connects to
    // nobody and its 10 messages reach nobody), exactly as the reference.
    PeerNode(const std::string& ip, int port, const std::vector<PeerInfo>& seeds);
    // Handle to peer `id` of a running simulation.
    PeerNode(std::shared_ptr<GossipNetwork> net, unsigned id);
    ~PeerNode();

    bool start();  // runs the (simulated) network to completion; false if the bootstrap failed
    void stop();
    bool isRunning() const;

    // -- extension: read-only views -----------------------------------------------
    unsigned id() const { return id_; }
    const std::string& ip() const { return ip_; }
    int port() const { return port_; }
    std::vector<PeerInfo> connectedPeers() const;                          // live out-edges
    std::unordered_map<std::string, MessageTracker> messageList() const;  // hash -> tracker
    std::shared_ptr<GossipNetwork> network() const { return net_; }

private:
    std::shared_ptr<GossipNetwork> net_;
    unsigned id_ = 0;
    std::string ip_;
    int port_ = 0;
};
