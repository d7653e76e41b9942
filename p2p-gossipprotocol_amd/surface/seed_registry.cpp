// seed_registry.cpp -- SeedNode: the registry side of the protocol.
#include <algorithm>
#include <fstream>
#include <iostream>

#include "gossip/formats.hpp"
#include "gossip/seed.hpp"

namespace {

// Minimal reader for the flat JSON objects the protocol exchanges.
bool json_field(const std::string& js, const std::string& key, std::string& out, bool& is_string) {
    const std::string pat = "\"" + key + "\"";
    size_t k = js.find(pat);
    if (k == std::string::npos) return false;
    size_t c = js.find(':', k + pat.size());
    if (c == std::string::npos) return false;
    size_t v = js.find_first_not_of(" \t\r\n", c + 1);
    if (v == std::string::npos) return false;
    if (js[v] == '"') {
        size_t e = js.find('"', v + 1);
        if (e == std::string::npos) return false;
        out = js.substr(v + 1, e - v - 1);
        is_string = true;
    } else {
        size_t e = js.find_first_of(",}", v);
        out = js.substr(v, e == std::string::npos ? std::string::npos : e - v);
        is_string = false;
    }
    return true;
}

}  // namespace

SeedNode::SeedNode(const std::string& ip, int port) : ip_(ip), port_(port) {}
SeedNode::~SeedNode() { stop(); }

bool SeedNode::start() {
    running_ = true;
    const std::string msg = "Seed node started on port " + std::to_string(port_);
    if (!logPath_.empty()) std::cout << msg << std::endl;
    log(msg);
    return true;
}

void SeedNode::stop() { running_ = false; }

// peerList[peer] = now (seed.cpp:153-156): a new key keeps the time of its first insertion (the key's
// lastSeen, which getPeerList reports, seed.cpp:169-177); a repeated registration only updates the mapped value
void SeedNode::addPeer(const PeerInfo& peer) {
    std::lock_guard<std::mutex> g(mu_);
    const auto now = std::chrono::system_clock::time_point(std::chrono::seconds(clock_));
    auto it = peers_.find(peer);
    if (it == peers_.end()) {
        PeerInfo key = peer;
        key.lastSeen = now;
        order_.push_back(key);
    }
    peers_[peer] = now;
}

void SeedNode::handleDeadNode(const std::string& deadIP, int deadPort) {
    std::lock_guard<std::mutex> g(mu_);
    PeerInfo dead{deadIP, deadPort, {}};
    if (peers_.erase(dead) > 0) {
        order_.erase(std::remove(order_.begin(), order_.end(), dead), order_.end());
        const std::string msg = "Removed dead peer: " + deadIP + ":" + std::to_string(deadPort);
        std::cout << msg << std::endl;  // unconditionally, as seed.cpp:164
        log(msg);
    }
}

std::vector<PeerInfo> SeedNode::getPeerList() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<PeerInfo> out;
    out.reserve(order_.size());
    for (const PeerInfo& p : order_) out.push_back(p);  // keys, with their first-insert lastSeen
    return out;
}

size_t SeedNode::size() {
    std::lock_guard<std::mutex> g(mu_);
    return peers_.size();
}

std::string SeedNode::handleRequest(const std::string& js) {
    std::string type, a, b;
    bool s1 = false, s2 = false, s3 = false;
    if (!json_field(js, "type", type, s1)) {
        log("Error handling client message: missing type");
        return "";
    }
    if (type == "register" && json_field(js, "ip", a, s2) && json_field(js, "port", b, s3)) {
        PeerInfo p{a, std::stoi(b), {}};
        addPeer(p);
        const std::string response = gossip::peer_list_json(getPeerList());
        log("Registered new peer: " + a + ":" + b);
        return response;
    }
    if (type == "dead_node" && json_field(js, "dead_ip", a, s2) && json_field(js, "dead_port", b, s3)) {
        handleDeadNode(a, std::stoi(b));
        log("Received dead node notification for: " + a + ":" + b);
        return "";
    }
    return "";
}

void SeedNode::setLogDir(const std::string& dir) {
    logPath_ = dir.empty() ? std::string() : dir + "/seed_" + std::to_string(port_) + "_output.txt";
}

void SeedNode::log(const std::string& message) {
    if (logPath_.empty()) return;
    std::ofstream f(logPath_, std::ios::app);
    if (f) f << gossip::seed_log_line(static_cast<std::time_t>(clock_), message);
}
