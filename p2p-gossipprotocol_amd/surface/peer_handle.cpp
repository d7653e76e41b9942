// peer_handle.cpp -- PeerNode handles and the Peer facade.
#include <iostream>

#include "gossip/formats.hpp"
#include "gossip/network.hpp"
#include "gossip/wrapper.hpp"

PeerNode::PeerNode(const std::string& ip, int port, const std::vector<PeerInfo>& seeds) : id_(0), ip_(ip), port_(port) {
    // A lone bootstrap: the first (and only) arrival of an empty network.
    SimOptions opt;
    opt.n_peers = 1;
    opt.graph = "ref_bootstrap";
    opt.addresses = {{ip, port}};
    opt.ping_every = 15;
    net_ = std::make_shared<GossipNetwork>(seeds, opt);
}

PeerNode::PeerNode(std::shared_ptr<GossipNetwork> net, unsigned id) : net_(std::move(net)), id_(id) {
    const PeerInfo p = net_->peerInfo(id);
    ip_ = p.ip;
    port_ = p.port;
}

PeerNode::~PeerNode() = default;

bool PeerNode::start() {
    if (!net_->start()) {
        std::cerr << "Failed to connect to minimum required seeds" << std::endl;  // peer.cpp:75
        return false;
    }
    return net_->run();
}

void PeerNode::stop() { net_->stop(); }
bool PeerNode::isRunning() const { return net_->isRunning(); }

std::vector<PeerInfo> PeerNode::connectedPeers() const {
    std::vector<PeerInfo> out;
    for (uint32_t c : net_->rowOf(id_))
        if (net_->edgeLive(id_, c)) out.push_back(net_->peerInfo(c));
    return out;
}

std::unordered_map<std::string, MessageTracker> PeerNode::messageList() const {
    std::unordered_map<std::string, MessageTracker> out;
    if (!net_->traced()) return out;
    for (uint32_t m = 0; m < net_->messages(); ++m) {
        if (net_->receiptRound(id_, m) < 0) continue;
        MessageTracker t;
        t.msg = net_->message(m);
        for (uint32_t c : net_->sentTo(id_, m)) {
            const PeerInfo p = net_->peerInfo(c);
            t.sentTo.insert({p.ip, p.port});
        }
        out.emplace(t.msg.hash, std::move(t));
    }
    return out;
}

Peer::Peer(const std::string& configFile) : config_(configFile) {
    net_ = std::make_shared<GossipNetwork>(config_, SimOptions::fromConfig(config_));
    node = std::make_unique<PeerNode>(net_, 0u);
}

Peer::~Peer() { stop(); }

void Peer::start() {
    if (node) node->start();
}

void Peer::stop() {
    if (node) node->stop();
}

bool Peer::isRunning() const { return node && node->isRunning(); }
