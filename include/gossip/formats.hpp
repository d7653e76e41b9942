// formats.hpp -- the reference's observable strings, produced from engine ids.
//
//   message hash  hex(SHA-256(content || timestamp || sourceIP))   peer.cpp:135-159
//   gossip JSON   {"content","hash","msg_number","source_ip","source_port","timestamp","type"}  peer.cpp:298-307
//   register      {"ip","port","type"}                              peer.cpp:176-180
//   peer_list     {"peers":[{"ip","lastSeen","port"},...],"type"}  seed.cpp:120-123, info.hpp:26-32
//   dead_node     {"dead_ip","dead_port","type"}                    seed.cpp:130-136 (never sent by the reference, F7)
//   peer log      ctime(t) + ": " + msg   (ctime keeps its '\n')    peer.cpp:125-133
//   seed log      ctime(t) + msg                                    seed.cpp:180-188
// JSON is compact with keys in sorted order, as nlohmann::json::dump() emits.
#pragma once

#include <cstdint>
#include <ctime>
#include <string>
#include <vector>

#include "gossip/info.hpp"

namespace gossip {

// Deterministic clock of the simulation: round r happens at kEpoch + r seconds
// (one round = one second of the reference's wall clock).
constexpr long long kEpochSeconds = 1740441600LL;  // 2025-02-25T00:00:00Z, the reference snapshot

struct PeerAddress {
    std::string ip;
    int port;
};

// Address of simulated peer `id`: loopback ports 5000.. for small networks
// (the README's "n terminals" case), 10.x.y.z:5000+ beyond that.
PeerAddress peer_address(uint64_t id, uint64_t n_peers);

std::string message_content(const PeerAddress& origin);                // "Message from <ip>:<port>"
std::string message_timestamp(uint32_t round);                         // 19-digit ns since epoch
std::string message_hash(const std::string& content, const std::string& timestamp, const std::string& source_ip);

std::string json_escape(const std::string& s);
std::string gossip_json(const std::string& content, const std::string& hash, int msg_number,
                        const std::string& source_ip, int source_port, const std::string& timestamp);
std::string register_json(const std::string& ip, int port);
std::string peer_list_json(const std::vector<PeerInfo>& peers);
std::string dead_node_json(const std::string& ip, int port);

std::string ctime_string(std::time_t t);                               // ctime(), '\n' included
std::string peer_log_line(std::time_t t, const std::string& msg);      // "<ctime>: <msg>\n"
std::string seed_log_line(std::time_t t, const std::string& msg);      // "<ctime><msg>\n"

}  // namespace gossip
