// ref_config_driver.cpp -- TEST INFRASTRUCTURE ONLY.
// Links the reference's own config.cpp (compiled where it lies under
// /root/reference by oracle/Makefile, output to oracle/_ref/) and prints what
// NetworkConfig(path) produces for each path given on the command line, one
// JSON object per line.  Used only by tests/golden/make_config_golden.py to
// pin the drop-in NetworkConfig against the real reference (config.cpp:1-182).
#include "config.hpp"
#include <cstdio>
#include <exception>
#include <string>

static std::string esc(const std::string& s) {
    std::string o;
    for (char c : s) {
        if (c == '"' || c == '\\') { o += '\\'; o += c; }
        else if (c == '\n') o += "\\n";
        else if (c == '\t') o += "\\t";
        else if (c == '\r') o += "\\r";
        else o += c;
    }
    return o;
}

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        try {
            NetworkConfig cfg(argv[i]);
            std::string seeds;
            for (const auto& s : cfg.getSeedNodes()) {
                if (!seeds.empty()) seeds += ",";
                seeds += "\"" + esc(s.toString()) + "\"";
            }
            std::printf("{\"ok\":true,\"seeds\":[%s],\"min_seeds\":%d,\"ping_interval\":%d,"
                        "\"message_interval\":%d,\"max_messages\":%d,\"max_missed_pings\":%d,"
                        "\"local_ip\":\"%s\",\"local_port\":%d,\"to_string\":\"%s\"}\n",
                        seeds.c_str(), cfg.getMinRequiredSeeds(), cfg.getPingInterval(),
                        cfg.getMessageInterval(), cfg.getMaxMessages(), cfg.getMaxMissedPings(),
                        esc(cfg.getLocalIP()).c_str(), cfg.getLocalPort(), esc(cfg.toString()).c_str());
        } catch (const NetworkConfig::ConfigException& e) {
            std::printf("{\"ok\":false,\"kind\":\"ConfigException\",\"what\":\"%s\"}\n", esc(e.what()).c_str());
        } catch (const std::exception& e) {
            std::printf("{\"ok\":false,\"kind\":\"std::exception\",\"what\":\"%s\"}\n", esc(e.what()).c_str());
        }
    }
    return 0;
}
