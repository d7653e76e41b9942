// network_config.cpp -- NetworkConfig for the drop-in surface.
// Behaviour pinned line-for-line against the reference's own config.cpp
// (compiled in oracle/_ref/, fixtures in tests/golden/config_cases.json).
#include "gossip/config.hpp"

#include <arpa/inet.h>

#include <algorithm>
#include <fstream>
#include <sstream>

namespace {

const char* const kBlank = " \t\r\n";

std::string strip(const std::string& s) {
    const size_t a = s.find_first_not_of(kBlank);
    if (a == std::string::npos) return std::string();
    return s.substr(a, s.find_last_not_of(kBlank) - a + 1);
}

bool ipv4(const std::string& s) {
    in_addr out{};
    return ::inet_pton(AF_INET, s.c_str(), &out) == 1;
}

bool port_ok(int p) { return 0 < p && p < 65536; }

// splitmix-style draw used by getRandomSeeds (deterministic per object)
unsigned long long mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

NetworkConfig::NodeInfo::NodeInfo() : ip(), port(0) {}
NetworkConfig::NodeInfo::NodeInfo(const std::string& i, int p) : ip(i), port(p) {}
bool NetworkConfig::NodeInfo::operator==(const NodeInfo& o) const { return port == o.port && ip == o.ip; }
std::string NetworkConfig::NodeInfo::toString() const { return ip + ":" + std::to_string(port); }

NetworkConfig::ConfigException::ConfigException(const std::string& m) : std::runtime_error("Configuration Error: " + m) {}

NetworkConfig::NetworkConfig(const std::string& configPath) : path_(configPath) {
    read();
    check();
}

void NetworkConfig::read() {
    std::ifstream in(path_);
    if (!in) throw ConfigException("Unable to open config file: " + path_);
    std::string raw;
    for (int lineNo = 1; std::getline(in, raw); ++lineNo) {
        const std::string line = strip(raw);
        if (line.empty() || line.front() == '#') continue;
        try {
            consume(line);
        } catch (const ConfigException& e) {
            throw ConfigException("Error at line " + std::to_string(lineNo) + ": " + e.what());
        }
    }
    if (seeds_.empty()) throw ConfigException("No valid seed nodes found in configuration");
    quorum_ = static_cast<int>(seeds_.size() / 2 + 1);
}

// One non-comment line: `key=value` (any '=' present) or `ip:port`.
void NetworkConfig::consume(const std::string& line) {
    const size_t eq = line.find('=');
    if (eq != std::string::npos) {
        const std::string key = strip(line.substr(0, eq));
        const std::string value = strip(line.substr(eq + 1));
        if (key.empty() || value.empty()) throw ConfigException("Invalid configuration format");
        static const std::pair<const char*, int NetworkConfig::*> known[] = {
            {"ping_interval", &NetworkConfig::pingInterval_},
            {"message_interval", &NetworkConfig::messageInterval_},
            {"max_messages", &NetworkConfig::maxMessages_},
            {"max_missed_pings", &NetworkConfig::maxMissedPings_},
        };
        for (const auto& k : known)
            if (key == k.first) this->*(k.second) = std::stoi(value);  // std::invalid_argument escapes, as in the reference
        extra_[key] = value;
        return;
    }
    const size_t colon = line.find(':');
    if (colon == std::string::npos || colon + 1 == line.size()) throw ConfigException("Invalid seed node format");
    const std::string ip = strip(line.substr(0, colon));
    const std::string portText = strip(line.substr(colon + 1));
    if (!ipv4(ip)) throw ConfigException("Invalid IP address: " + ip);
    int port = 0;
    bool good = true;
    try {
        port = std::stoi(portText);  // lenient: "8000abc" -> 8000, like the reference
    } catch (const std::exception&) {
        good = false;
    }
    if (!good || !port_ok(port)) throw ConfigException("Invalid port format: " + portText);
    seeds_.emplace_back(ip, port);
}

void NetworkConfig::check() const {
    if (pingInterval_ <= 0) throw ConfigException("Ping interval must be positive");
    if (messageInterval_ <= 0) throw ConfigException("Message interval must be positive");
    if (maxMessages_ <= 0) throw ConfigException("Maximum message count must be positive");
    if (maxMissedPings_ <= 0) throw ConfigException("Maximum missed pings must be positive");
    for (const NodeInfo& s : seeds_)
        if (!ipv4(s.ip) || !port_ok(s.port)) throw ConfigException("Invalid seed node configuration: " + s.toString());
    std::vector<std::pair<std::string, int>> keys;
    keys.reserve(seeds_.size());
    for (const NodeInfo& s : seeds_) keys.emplace_back(s.ip, s.port);
    std::sort(keys.begin(), keys.end());
    if (std::adjacent_find(keys.begin(), keys.end()) != keys.end())
        throw ConfigException("Duplicate seed nodes found in configuration");
}

const std::vector<NetworkConfig::NodeInfo>& NetworkConfig::getSeedNodes() const { return seeds_; }
std::string NetworkConfig::getLocalIP() const { return localIp_; }
int NetworkConfig::getLocalPort() const { return localPort_; }
int NetworkConfig::getMinRequiredSeeds() const { return quorum_; }
int NetworkConfig::getPingInterval() const { return pingInterval_; }
int NetworkConfig::getMessageInterval() const { return messageInterval_; }
int NetworkConfig::getMaxMessages() const { return maxMessages_; }
int NetworkConfig::getMaxMissedPings() const { return maxMissedPings_; }

std::vector<NetworkConfig::NodeInfo> NetworkConfig::getRandomSeeds(int count) const {
    if (count > static_cast<int>(seeds_.size())) throw ConfigException("Requested more seeds than available");
    std::vector<NodeInfo> out = seeds_;
    for (size_t i = out.size(); i > 1; --i) {
        const unsigned long long r = mix(++shuffleCounter_ ^ 0x5EEDull);
        std::swap(out[i - 1], out[r % i]);
    }
    out.resize(count < 0 ? 0 : static_cast<size_t>(count));
    return out;
}

std::string NetworkConfig::toString() const {
    std::ostringstream os;
    os << "Network Configuration:\n----------------------\n";
    os << "Seed Nodes (" << seeds_.size() << "):\n";
    for (const NodeInfo& s : seeds_) os << " " << s.toString() << "\n";
    os << "Minimum Required Seeds: " << quorum_ << "\n"
       << "Network Parameters:\n"
       << " Ping Interval: " << pingInterval_ << " seconds\n"
       << " Message Interval: " << messageInterval_ << " seconds\n"
       << " Max Messages: " << maxMessages_ << "\n"
       << " Max Missed Pings: " << maxMissedPings_ << "\n";
    return os.str();
}

bool NetworkConfig::hasKey(const std::string& key) const { return extra_.count(key) != 0; }

std::string NetworkConfig::getString(const std::string& key, const std::string& fallback) const {
    auto it = extra_.find(key);
    return it == extra_.end() ? fallback : it->second;
}

long long NetworkConfig::getInt(const std::string& key, long long fallback) const {
    auto it = extra_.find(key);
    if (it == extra_.end()) return fallback;
    return std::stoll(it->second, nullptr, 0);
}
