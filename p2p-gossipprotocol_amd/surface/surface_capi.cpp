// surface_capi.cpp -- extern "C" probes of the drop-in surface for the test
// harness (ctypes): NetworkConfig outcomes and the reference string formats.
#include <cstring>
#include <exception>
#include <string>

#include <sstream>

#include "gossip/config.hpp"
#include "gossip/formats.hpp"
#include "gossip/seed.hpp"

namespace {

int put(const std::string& s, char* out, size_t cap) {
    if (!out || cap == 0) return -1;
    const size_t k = std::min(cap - 1, s.size());
    std::memcpy(out, s.data(), k);
    out[k] = 0;
    return s.size() < cap ? 0 : -1;
}

}  // namespace

extern "C" {

// JSON object in the shape of oracle/ref_config_driver's output.
int gossip_surface_netcfg(const char* path, char* out, size_t cap) {
    std::string js;
    try {
        NetworkConfig c(path);
        std::string seeds;
        for (const auto& s : c.getSeedNodes()) seeds += (seeds.empty() ? "" : ",") + gossip::json_escape(s.toString());
        js = "{\"ok\":true,\"seeds\":[" + seeds + "],\"min_seeds\":" + std::to_string(c.getMinRequiredSeeds()) +
             ",\"ping_interval\":" + std::to_string(c.getPingInterval()) +
             ",\"message_interval\":" + std::to_string(c.getMessageInterval()) +
             ",\"max_messages\":" + std::to_string(c.getMaxMessages()) +
             ",\"max_missed_pings\":" + std::to_string(c.getMaxMissedPings()) +
             ",\"local_ip\":" + gossip::json_escape(c.getLocalIP()) + ",\"local_port\":" + std::to_string(c.getLocalPort()) +
             ",\"to_string\":" + gossip::json_escape(c.toString()) + "}";
    } catch (const NetworkConfig::ConfigException& e) {
        js = "{\"ok\":false,\"kind\":\"ConfigException\",\"what\":" + gossip::json_escape(e.what()) + "}";
    } catch (const std::exception& e) {
        js = "{\"ok\":false,\"kind\":\"std::exception\",\"what\":" + gossip::json_escape(e.what()) + "}";
    }
    return put(js, out, cap);
}

int gossip_surface_message(const char* ip, int port, unsigned round, int msg_number, char* out, size_t cap) {
    const std::string content = gossip::message_content({ip, port});
    const std::string ts = gossip::message_timestamp(round);
    const std::string h = gossip::message_hash(content, ts, ip);
    return put(gossip::gossip_json(content, h, msg_number, ip, port, ts), out, cap);
}

int gossip_surface_hash(const char* content, const char* timestamp, const char* ip, char* out, size_t cap) {
    return put(gossip::message_hash(content, timestamp, ip), out, cap);
}

int gossip_surface_register(const char* ip, int port, char* out, size_t cap) {
    return put(gossip::register_json(ip, port), out, cap);
}

int gossip_surface_dead_node(const char* ip, int port, char* out, size_t cap) {
    return put(gossip::dead_node_json(ip, port), out, cap);
}

// A SeedNode driven by requests, one per line "<unix seconds> <json>" (the seed's clock, then
// handleRequest); out gets each request's response (empty for dead_node) on a line of its own.
int gossip_surface_seed(const char* ops, char* out, size_t cap) {
    try {
        SeedNode seed("127.0.0.1", 8000);
        std::istringstream in(ops ? ops : "");
        std::string line, res;
        while (std::getline(in, line)) {
            const size_t sp = line.find(' ');
            if (sp == std::string::npos) continue;
            seed.setClock(std::stoll(line.substr(0, sp)));
            res += seed.handleRequest(line.substr(sp + 1)) + "\n";
        }
        return put(res, out, cap);
    } catch (const std::exception&) {
        return -2;
    }
}

// gossip_json from every field (a received message's bytes rebuilt from what it carries)
int gossip_surface_gossip_json(const char* content, const char* hash, int msg_number, const char* ip, int port,
                               const char* timestamp, char* out, size_t cap) {
    return put(gossip::gossip_json(content, hash, msg_number, ip, port, timestamp), out, cap);
}

// peer_list_json of entries "<ip> <port> <lastSeen>", one per line, in the given order
int gossip_surface_peer_list(const char* entries, char* out, size_t cap) {
    std::vector<PeerInfo> peers;
    std::istringstream in(entries ? entries : "");
    std::string ip;
    int port = 0;
    long long t = 0;
    while (in >> ip >> port >> t)
        peers.push_back(PeerInfo{ip, port, std::chrono::system_clock::time_point(std::chrono::seconds(t))});
    return put(gossip::peer_list_json(peers), out, cap);
}

// gossip_surface_seed with the seed's log: start() and every request logged to <logdir>/seed_8000_output.txt
int gossip_surface_seed_logged(const char* ops, const char* logdir, char* out, size_t cap) {
    try {
        SeedNode seed("127.0.0.1", 8000);
        std::istringstream in(ops ? ops : "");
        std::string line, res;
        bool started = false;
        while (std::getline(in, line)) {
            const size_t sp = line.find(' ');
            if (sp == std::string::npos) continue;
            seed.setClock(std::stoll(line.substr(0, sp)));
            if (!started) {
                seed.setLogDir(logdir ? logdir : "");
                seed.start();
                started = true;
            }
            res += seed.handleRequest(line.substr(sp + 1)) + "\n";
        }
        return put(res, out, cap);
    } catch (const std::exception&) {
        return -2;
    }
}

int gossip_surface_log(int seed_style, long long t, const char* msg, char* out, size_t cap) {
    return put(seed_style ? gossip::seed_log_line((std::time_t)t, msg) : gossip::peer_log_line((std::time_t)t, msg), out,
               cap);
}

}  // extern "C"
