// formats.cpp -- reference wire/log strings (see gossip/formats.hpp).
#include "gossip/formats.hpp"

#include <openssl/evp.h>

#include <cstdio>
#include <stdexcept>

namespace gossip {

PeerAddress peer_address(uint64_t id, uint64_t n_peers) {
    if (n_peers <= 60000) return {"127.0.0.1", static_cast<int>(5000 + id)};
    char buf[32];
    std::snprintf(buf, sizeof buf, "10.%u.%u.%u", (unsigned)((id >> 16) & 255), (unsigned)((id >> 8) & 255),
                  (unsigned)(id & 255));
    return {buf, static_cast<int>(5000 + (id >> 24))};
}

std::string message_content(const PeerAddress& o) { return "Message from " + o.ip + ":" + std::to_string(o.port); }

std::string message_timestamp(uint32_t round) {
    return std::to_string((kEpochSeconds + (long long)round) * 1000000000LL);
}

std::string message_hash(const std::string& content, const std::string& timestamp, const std::string& source_ip) {
    const std::string data = content + timestamp + source_ip;
    unsigned char md[EVP_MAX_MD_SIZE];
    unsigned int len = 0;
    EVP_MD_CTX* ctx = EVP_MD_CTX_new();
    if (!ctx) throw std::runtime_error("EVP_MD_CTX_new failed");
    EVP_DigestInit_ex(ctx, EVP_sha256(), nullptr);
    EVP_DigestUpdate(ctx, data.data(), data.size());
    EVP_DigestFinal_ex(ctx, md, &len);
    EVP_MD_CTX_free(ctx);
    static const char* hex = "0123456789abcdef";
    std::string out(2 * len, '0');
    for (unsigned i = 0; i < len; ++i) {
        out[2 * i] = hex[md[i] >> 4];
        out[2 * i + 1] = hex[md[i] & 15];
    }
    return out;
}

std::string json_escape(const std::string& s) {
    std::string o = "\"";
    for (unsigned char c : s) {
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            case '\b': o += "\\b"; break;
            case '\f': o += "\\f"; break;
            default:
                if (c < 0x20) {
                    char b[8];
                    std::snprintf(b, sizeof b, "\\u%04x", c);
                    o += b;
                } else {
                    o += static_cast<char>(c);
                }
        }
    }
    return o + "\"";
}

std::string gossip_json(const std::string& content, const std::string& hash, int msg_number,
                        const std::string& source_ip, int source_port, const std::string& timestamp) {
    return "{\"content\":" + json_escape(content) + ",\"hash\":" + json_escape(hash) +
           ",\"msg_number\":" + std::to_string(msg_number) + ",\"source_ip\":" + json_escape(source_ip) +
           ",\"source_port\":" + std::to_string(source_port) + ",\"timestamp\":" + json_escape(timestamp) +
           ",\"type\":\"gossip\"}";
}

std::string register_json(const std::string& ip, int port) {
    return "{\"ip\":" + json_escape(ip) + ",\"port\":" + std::to_string(port) + ",\"type\":\"register\"}";
}

std::string peer_list_json(const std::vector<PeerInfo>& peers) {
    std::string o = "{\"peers\":[";
    for (size_t i = 0; i < peers.size(); ++i) {
        if (i) o += ",";
        const long long seen = (long long)std::chrono::system_clock::to_time_t(peers[i].lastSeen);
        o += "{\"ip\":" + json_escape(peers[i].ip) + ",\"lastSeen\":" + std::to_string(seen) +
             ",\"port\":" + std::to_string(peers[i].port) + "}";
    }
    return o + "],\"type\":\"peer_list\"}";
}

std::string dead_node_json(const std::string& ip, int port) {
    return "{\"dead_ip\":" + json_escape(ip) + ",\"dead_port\":" + std::to_string(port) + ",\"type\":\"dead_node\"}";
}

std::string ctime_string(std::time_t t) {
    char buf[64];
    std::tm tm{};
    gmtime_r(&t, &tm);  // the simulation clock is UTC
    std::strftime(buf, sizeof buf, "%a %b %e %H:%M:%S %Y\n", &tm);
    return buf;
}

std::string peer_log_line(std::time_t t, const std::string& msg) { return ctime_string(t) + ": " + msg + "\n"; }
std::string seed_log_line(std::time_t t, const std::string& msg) { return ctime_string(t) + msg + "\n"; }

}  // namespace gossip
