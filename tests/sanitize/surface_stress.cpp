// surface_stress.cpp -- CPU sanitizer harness for the drop-in C++ surface
// (TSan/ASan on the host code).  Built by
// tests/sanitize/Makefile under ThreadSanitizer and under Address+UB
// sanitizers; run by tests/test_sanitizers.py.
//
// The reference's seed and peer are thread-per-connection (seed.cpp:64-79,
// peer.cpp:86-101) with a stop() called from a signal handler (main.cpp:14-22);
// the surface keeps that contract, so the same calls are made concurrently
// here: registrations, dead-node reports and peer-list reads on one SeedNode
// from several threads; start/stop/isRunning, clock and log from another;
// NetworkConfig parses and the wire/log formatters on every thread.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "gossip/config.hpp"
#include "gossip/formats.hpp"
#include "gossip/seed.hpp"

int main(int argc, char** argv) {
    const std::string cfg_path = argc > 1 ? argv[1] : "tests/golden/network.txt";
    SeedNode seed("192.168.1.100", 8000);
    seed.start();
    std::atomic<bool> done{false};
    std::atomic<long> bad{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t) {
        ts.emplace_back([&, t] {
            for (int i = 0; i < 400; ++i) {
                const int port = 5000 + t * 1000 + i;
                const std::string reply = seed.handleRequest(gossip::register_json("127.0.0.1", port));
                if (reply.find("\"type\":\"peer_list\"") == std::string::npos) bad++;
                if (i % 3 == 0) seed.handleRequest(gossip::dead_node_json("127.0.0.1", port));
                if (i % 50 == 1) {  // (this thread's peer i is registered and not reported)
                    const std::vector<PeerInfo> l = seed.getPeerList();
                    if (l.empty()) bad++;
                    NetworkConfig cfg(cfg_path);
                    if (cfg.getSeedNodes().size() != 20) bad++;
                }
                const std::string h = gossip::message_hash("Message from 127.0.0.1:" + std::to_string(port),
                                                           gossip::message_timestamp(i), "127.0.0.1");
                if (h.size() != 64) bad++;
            }
        });
    }
    ts.emplace_back([&] {  // the signal-handler side: stop / restart / status, and the seed's clock
        long k = 0;
        while (!done.load()) {
            seed.setClock(1740441600LL + (k++));
            if (k % 64 == 0) seed.stop();
            if (k % 64 == 32) seed.start();
            (void)seed.isRunning();
            (void)seed.size();
            std::this_thread::yield();
        }
    });
    for (int t = 0; t < 4; ++t) ts[t].join();
    done = true;
    ts.back().join();
    const size_t left = seed.size();
    std::printf("surface_stress: %zu peers registered, %ld bad replies\n", left, bad.load());
    return bad.load() == 0 && left == 4 * 400 - 4 * 134 ? 0 : 1;
}
