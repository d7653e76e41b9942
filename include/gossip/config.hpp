// config.hpp -- drop-in NetworkConfig (reference: config.hpp:7-57, config.cpp:1-182).
//
// Same class name, nested types, getters, exception type and messages as the
// reference, so code written against the reference compiles unchanged:
//   * `ip:port` lines are seeds, `key=value` lines set ping_interval,
//     message_interval, max_messages, max_missed_pings; `#` comments and
//     blank lines are skipped after trimming " \t\r\n";
//   * errors are NetworkConfig::ConfigException ("Configuration Error: ..."),
//     line errors re-wrapped as "Error at line N: ..." (config.cpp:68-69);
//     a non-numeric value of a known key escapes as std::invalid_argument
//     ("stoi"), exactly like config.cpp:93-96.
// Extension (behaviour-neutral for reference files): every key=value pair is
// also kept verbatim, so simulation keys (n_peers, rng_seed, graph, ...) can
// live in the same network.txt -- the reference ignores unknown keys too.
#pragma once

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

class NetworkConfig {
public:
    struct NodeInfo {
        std::string ip;
        int port;

        NodeInfo();
        NodeInfo(const std::string& ip, int port);
        bool operator==(const NodeInfo& other) const;
        std::string toString() const;
    };

    class ConfigException : public std::runtime_error {
    public:
        explicit ConfigException(const std::string& message);
    };

    NetworkConfig(const std::string& configPath);

    const std::vector<NodeInfo>& getSeedNodes() const;
    std::string getLocalIP() const;
    int getLocalPort() const;
    int getMinRequiredSeeds() const;
    int getPingInterval() const;
    int getMessageInterval() const;
    int getMaxMessages() const;
    int getMaxMissedPings() const;

    std::vector<NodeInfo> getRandomSeeds(int count) const;
    std::string toString() const;

    // -- extension: raw key=value pairs (last one wins) ----------------------
    bool hasKey(const std::string& key) const;
    std::string getString(const std::string& key, const std::string& fallback) const;
    long long getInt(const std::string& key, long long fallback) const;

private:
    std::string path_;
    std::vector<NodeInfo> seeds_;
    int quorum_ = 0;
    int pingInterval_ = 13;     // config.cpp:34
    int messageInterval_ = 5;   // config.cpp:35
    int maxMessages_ = 10;      // config.cpp:36
    int maxMissedPings_ = 3;    // config.cpp:37
    std::string localIp_ = "192.168.99.96";  // config.cpp:38
    int localPort_ = 5000;                   // config.cpp:39
    std::map<std::string, std::string> extra_;
    mutable unsigned long long shuffleCounter_ = 0;

    void read();
    void consume(const std::string& line);
    void check() const;
};
