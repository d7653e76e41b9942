// ref_registry_driver.cpp -- TEST INFRASTRUCTURE ONLY.
// Drives the reference's own SeedNode registry (seed.cpp:153-178) and PeerInfo's JSON serialiser (info.hpp:23-39,
// nlohmann/json 3.1.1 from the image) through a script on stdin, one command per line:
//   add <ip> <port> <lastSeen seconds>   SeedNode::addPeer(PeerInfo{ip, port, lastSeen})
//   dead <ip> <port>                     SeedNode::handleDeadNode(ip, port)
//   list                                 the register reply seed.cpp:120-123 builds: {"peers":getPeerList(),"type":..}
//   peer <ip> <port> <lastSeen seconds>  json(PeerInfo).dump()
// Each result is printed as "@<json>" (the seed's own stdout lines, e.g. "Removed dead peer", pass through);
// its log goes to seed_<port>_output.txt in the working directory.  Used only by
// tests/golden/make_ref_wire_golden.py.
#include "seed.hpp"
#include <nlohmann/json.hpp>
#include <iostream>
#include <sstream>
#include <string>

using json = nlohmann::json;

int main() {
    SeedNode seed("127.0.0.1", 7999);
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string cmd, ip;
        int port = 0;
        long long t = 0;
        in >> cmd;
        if (cmd == "add" && (in >> ip >> port >> t)) {
            seed.addPeer(PeerInfo{ip, port, std::chrono::system_clock::time_point(std::chrono::seconds(t))});
            std::cout << "@{}" << std::endl;
        } else if (cmd == "dead" && (in >> ip >> port)) {
            seed.handleDeadNode(ip, port);
            std::cout << "@{}" << std::endl;
        } else if (cmd == "list") {
            json response;
            response["type"] = "peer_list";
            response["peers"] = seed.getPeerList();
            std::cout << "@" << response.dump() << std::endl;
        } else if (cmd == "peer" && (in >> ip >> port >> t)) {
            json j = PeerInfo{ip, port, std::chrono::system_clock::time_point(std::chrono::seconds(t))};
            std::cout << "@" << j.dump() << std::endl;
        } else {
            std::cout << "@error" << std::endl;
        }
    }
    return 0;
}
