// info.hpp -- drop-in PeerInfo / PeerInfoHash (reference: info.hpp:6-39).
// The reference serialises PeerInfo with nlohmann::json (info.hpp:23-39); the
// surface does not depend on it: the wire form {"ip","lastSeen","port"} (sorted
// keys, compact) is produced by gossip/formats.hpp, byte-exact against the
// reference's own serialiser (tests/test_ref_wire.py).
#pragma once

#include <chrono>
#include <functional>
#include <string>

struct PeerInfo {
    std::string ip;
    int port;
    std::chrono::system_clock::time_point lastSeen;

    bool operator==(const PeerInfo& other) const { return ip == other.ip && port == other.port; }
};

struct PeerInfoHash {
    size_t operator()(const PeerInfo& p) const { return std::hash<std::string>()(p.ip) ^ std::hash<int>()(p.port); }
};
