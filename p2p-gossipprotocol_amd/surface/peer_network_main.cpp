// peer_network_main.cpp -- gossip_peer_network <config_file> [--logs DIR]
// Drop-in for the reference CLI (main.cpp:29-78): same messages, same
// SIGINT/SIGTERM handling, same exit codes; one invocation runs the whole
// simulated network that network.txt (+ simulation keys) describes, and
// prints one JSON summary line per round and a final summary.
#include <csignal>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>

#include "gossip/config.hpp"
#include "gossip/wrapper.hpp"

static std::unique_ptr<Peer> g_peer;

static void on_signal(int signum) {
    std::cout << "\nReceived signal " << signum << std::endl;
    std::cout << "Initiating graceful shutdown..." << std::endl;
    if (g_peer) g_peer->stop();
}

static void usage(const char* prog) {
    std::cout << "Usage: " << prog << " <config_file>" << std::endl;
    std::cout << "Example: " << prog << " config.txt" << std::endl;
}

int main(int argc, char* argv[]) {
    if (argc < 2) {
        std::cerr << "Error: Invalid number of arguments" << std::endl;
        usage(argv[0]);
        return 1;
    }
    std::string logs;
    for (int i = 2; i + 1 < argc; ++i)
        if (std::strcmp(argv[i], "--logs") == 0) logs = argv[i + 1];
    std::signal(SIGINT, on_signal);
    std::signal(SIGTERM, on_signal);
    try {
        std::cout << "Initializing peer node..." << std::endl;
        const std::string configFile = argv[1];
        try {
            NetworkConfig config(configFile);
            std::cout << "Configuration loaded successfully:" << std::endl;
            std::cout << config.toString() << std::endl;
        } catch (const NetworkConfig::ConfigException& e) {
            std::cerr << "Configuration error: " << e.what() << std::endl;
            return 1;
        }
        g_peer = std::make_unique<Peer>(configFile);
        if (!logs.empty()) const_cast<SimOptions&>(g_peer->network()->options()).log_dir = logs;
        std::cout << "Starting peer node..." << std::endl;
        g_peer->start();
        auto net = g_peer->network();
        unsigned long long deliveries = 0, receipts = 0;
        for (const gossip_round_stats& s : net->rounds()) {
            deliveries += s.deliveries;
            receipts += s.new_receipts;
            std::cout << "{\"round\":" << s.round << ",\"frontier\":" << s.frontier << ",\"deliveries\":" << s.deliveries
                      << ",\"new_receipts\":" << s.new_receipts << ",\"died\":" << s.died << ",\"reports\":" << s.reports
                      << ",\"covered\":" << s.covered << "}" << std::endl;
        }
        std::cout << "{\"summary\":true,\"peers\":" << net->size() << ",\"messages\":" << net->messages()
                  << ",\"rounds\":" << net->rounds().size() << ",\"deliveries\":" << deliveries
                  << ",\"new_receipts\":" << receipts << ",\"reports\":" << net->reports().size() << "}" << std::endl;
        std::cout << "Shutting down peer node..." << std::endl;
        g_peer->stop();
        const bool ok = net->finished();
        g_peer.reset();
        std::cout << "Peer node shutdown complete" << std::endl;
        return ok ? 0 : 1;
    } catch (const std::exception& e) {
        std::cerr << "Fatal error: " << e.what() << std::endl;
        if (g_peer) {
            g_peer->stop();
            g_peer.reset();
        }
        return 1;
    }
}
