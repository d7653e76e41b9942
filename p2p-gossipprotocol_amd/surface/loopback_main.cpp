// loopback_main.cpp -- gossip_loopback: the build's real-socket loopback
// harness.
//
// Runs a small overlay as real TCP peers on 127.0.0.1 inside one process: S
// seed listeners (SeedNode::handleRequest behind a socket), one listener per
// peer, one TCP connection per overlay edge, and the reference's wire
// protocol end to end:
//   registration  PeerNode::start -> connectToSeed (peer.cpp:62-78,161-211):
//                 peers start in id order; peer i sends {"type":"register"} to
//                 seeds 0, 1, ... until q = S/2+1 of them answered with a
//                 parseable peer_list (seed.cpp:109-129).  --list-cap B reads at
//                 most B bytes of a response, the reference's 4 KB recv
//                 (peer.cpp:188-190, F10): a longer list fails that seed, and a
//                 peer with fewer than q successes does not start.
//   edges         the out-edges are the given CSR rows (the engine's overlay),
//                 connected once, as selectAndConnectPeers does (peer.cpp:242-250);
//                 edges to peers that did not start are refused.
//   gossip        messageGenerationLoop (peer.cpp:357-379) builds content,
//                 timestamp, hash (SHA-256, peer.cpp:135-159) and the gossip
//                 JSON; handleClient (peer.cpp:255-295) parses it, recomputes
//                 the hash, dedups on it, logs "Received new message", and
//                 broadcastMessage (peer.cpp:297-318) sends it on every
//                 out-connection, counting sentTo.
// The "fixed" parts: messages are newline-framed (the reference's unframed
// recv can split or merge them, F2) and one event loop replaces the
// thread-per-connection locking that deadlocks (F3).  Every received line must
// re-serialise to the identical bytes and carry the recomputed hash.
//
// Without churn the end state is independent of delivery order, so it must
// equal the round model's: every peer's message set, and
// sum |sentTo| = the engine's total deliveries, sum of new receipts.
//
// usage: gossip_loopback <input> [--seeds S] [--list-cap BYTES] [--log-dir DIR]
// input (whitespace separated): n m, row_ptr[n+1], col[m], n_msgs,
//   n_msgs x (origin inject_round msg_number)
// output (stdout): "started K", "deliveries D", "receipts R", "errors E",
//   then "seen v m0 m1 ..." per started peer (message indices, sorted).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "gossip/formats.hpp"
#include "gossip/seed.hpp"

namespace {

[[noreturn]] void die(const std::string& what) {
    std::cerr << "gossip_loopback: " << what << (errno ? std::string(": ") + std::strerror(errno) : "") << std::endl;
    std::exit(2);
}

int listen_socket(uint16_t* port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) die("socket");
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = 0;  // ephemeral: the logical address (gossip::peer_address) is what the messages carry
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0) die("bind");
    if (listen(fd, 4096) < 0) die("listen");
    socklen_t len = sizeof a;
    getsockname(fd, (sockaddr*)&a, &len);
    *port = ntohs(a.sin_port);
    return fd;
}

int connect_to(uint16_t port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) die("socket");
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(port);
    if (connect(fd, (sockaddr*)&a, sizeof a) < 0) die("connect");
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    return fd;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

void write_all(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        const ssize_t k = write(fd, s.data() + off, s.size() - off);
        if (k < 0) die("write");
        off += (size_t)k;
    }
}

std::string read_line(int fd) {  // blocking, up to '\n' (registration: one message per connection)
    std::string s;
    char b[65536];
    while (true) {
        const ssize_t k = read(fd, b, sizeof b);
        if (k < 0) die("read");
        if (k == 0) return s;
        s.append(b, (size_t)k);
        const size_t nl = s.find('\n');
        if (nl != std::string::npos) return s.substr(0, nl);
    }
}

// Flat JSON object reader for the protocol's messages (string and integer
// values; the escapes json_escape emits).
bool json_get(const std::string& js, const std::string& key, std::string* out) {
    const std::string pat = "\"" + key + "\":";
    const size_t k = js.find(pat);
    if (k == std::string::npos) return false;
    size_t v = k + pat.size();
    if (v >= js.size()) return false;
    std::string o;
    if (js[v] == '"') {
        for (++v; v < js.size() && js[v] != '"'; ++v) {
            if (js[v] != '\\') {
                o += js[v];
                continue;
            }
            if (++v >= js.size()) return false;
            switch (js[v]) {
                case 'n': o += '\n'; break;
                case 'r': o += '\r'; break;
                case 't': o += '\t'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'u':
                    if (v + 4 >= js.size()) return false;
                    o += (char)std::strtol(js.substr(v + 1, 4).c_str(), nullptr, 16);
                    v += 4;
                    break;
                default: o += js[v];
            }
        }
        if (v >= js.size()) return false;
    } else {
        const size_t e = js.find_first_of(",}]", v);
        o = js.substr(v, e == std::string::npos ? std::string::npos : e - v);
    }
    *out = o;
    return true;
}

struct Conn {
    int fd;
    int owner;      // peer that reads (incoming) or writes (outgoing) this socket
    bool outgoing;  // outgoing: this peer's out-edge; written only
    std::string buf;
    size_t off = 0;
};

struct Tracker {  // MessageTracker (peer.hpp:23-26)
    int index;
    std::set<int> sent_to;
};

struct Peer {
    bool started = false;
    uint16_t port = 0;  // real (ephemeral) listening port
    int listen_fd = -1;
    gossip::PeerAddress addr;
    std::vector<int> out;  // Conn indices of the out-edges, in row order
    std::vector<int> out_peer;
    std::unordered_map<std::string, Tracker> messages;  // messageList keyed by hash
    std::vector<std::string> log;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::cerr << "usage: gossip_loopback <input> [--seeds S] [--list-cap BYTES] [--log-dir DIR]" << std::endl;
        return 2;
    }
    int n_seeds = 20;
    size_t list_cap = 0;
    std::string log_dir;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--seeds" && i + 1 < argc) n_seeds = std::atoi(argv[++i]);
        else if (a == "--list-cap" && i + 1 < argc) list_cap = std::strtoull(argv[++i], nullptr, 0);
        else if (a == "--log-dir" && i + 1 < argc) log_dir = argv[++i];
        else die("bad argument " + a);
    }
    std::ifstream in(argv[1]);
    uint64_t n = 0, m = 0;
    if (!(in >> n >> m) || n == 0 || n > 4096 || m > 200000) die("bad input header (n <= 4096, m <= 200000)");
    std::vector<uint64_t> rp(n + 1);
    std::vector<uint32_t> col(m);
    for (auto& x : rp) in >> x;
    for (auto& x : col) in >> x;
    uint32_t n_msgs = 0;
    in >> n_msgs;
    struct Gen {
        uint32_t origin, round;
        int number;
    };
    std::vector<Gen> gen(n_msgs);
    for (auto& g : gen) in >> g.origin >> g.round >> g.number;
    if (!in) die("truncated input");
    for (uint64_t v = 0; v < n; ++v)
        if (rp[v] > rp[v + 1] || rp[v + 1] > m) die("bad row_ptr");
    for (uint32_t c : col)
        if (c >= n) die("bad col");

    // ---- seeds: SeedNode registries behind real listeners ----
    const int q = n_seeds / 2 + 1;  // peer.cpp:64
    std::vector<SeedNode*> seeds;
    std::vector<int> seed_fd(n_seeds);
    std::vector<uint16_t> seed_port(n_seeds);
    for (int s = 0; s < n_seeds; ++s) {
        seeds.push_back(new SeedNode("127.0.0.1", 8000 + s));
        if (!log_dir.empty()) seeds[s]->setLogDir(log_dir);
        seeds[s]->setClock(gossip::kEpochSeconds);
        seeds[s]->start();
        seed_fd[s] = listen_socket(&seed_port[s]);
    }

    std::vector<Peer> peers(n);
    uint64_t errors = 0;
    // ---- registration, peers in id order (PeerNode::start, peer.cpp:62-78) ----
    for (uint64_t v = 0; v < n; ++v) {
        Peer& p = peers[v];
        p.addr = gossip::peer_address(v, n);
        int ok = 0;
        for (int s = 0; s < n_seeds && ok < q; ++s) {
            const int c = connect_to(seed_port[s]);
            write_all(c, gossip::register_json(p.addr.ip, p.addr.port) + "\n");
            // seed side (seed.cpp:92-129): accept, read the request, answer
            const int a = accept(seed_fd[s], nullptr, nullptr);
            if (a < 0) die("accept (seed)");
            const std::string reply = seeds[s]->handleRequest(read_line(a));
            write_all(a, reply + "\n");
            close(a);
            // peer side (peer.cpp:186-210): one bounded read, parse the list
            const std::string resp = read_line(c);
            close(c);
            if (list_cap && resp.size() > list_cap) continue;  // truncated JSON: the parse fails
            std::string type;
            if (!json_get(resp, "type", &type) || type != "peer_list") {
                ++errors;
                continue;
            }
            // the list is the seed's registry in registration order, ending with v
            const std::string last = "{\"ip\":\"" + p.addr.ip + "\"";
            const size_t k = resp.rfind("{\"ip\":");
            if (k == std::string::npos || resp.compare(k, last.size(), last) != 0 ||
                resp.find("\"port\":" + std::to_string(p.addr.port) + "}", k) == std::string::npos)
                ++errors;
            ++ok;
        }
        if (ok < q) continue;  // "Failed to connect to minimum required seeds": stop()
        p.started = true;
        p.listen_fd = listen_socket(&p.port);
        set_nonblock(p.listen_fd);
        p.log.push_back(gossip::peer_log_line(gossip::kEpochSeconds, "Peer node started on port " +
                                                                          std::to_string(p.addr.port)));
    }

    // ---- overlay edges: one connection per out-edge ----
    std::vector<Conn> conns;
    auto accept_pending = [&](uint64_t v) {
        while (true) {
            const int a = accept(peers[v].listen_fd, nullptr, nullptr);
            if (a < 0) {
                if (errno == EAGAIN || errno == EWOULDBLOCK) {
                    errno = 0;
                    return;
                }
                die("accept");
            }
            set_nonblock(a);
            conns.push_back(Conn{a, (int)v, false, {}, 0});
        }
    };
    uint64_t refused = 0;
    for (uint64_t u = 0; u < n; ++u) {
        if (!peers[u].started) continue;
        for (uint64_t e = rp[u]; e < rp[u + 1]; ++e) {
            const uint32_t v = col[e];
            if (v == u) continue;
            if (!peers[v].started) {  // connect() to a peer that is not listening fails
                ++refused;
                continue;
            }
            const int fd = connect_to(peers[v].port);
            set_nonblock(fd);
            peers[u].out.push_back((int)conns.size());
            peers[u].out_peer.push_back((int)v);
            conns.push_back(Conn{fd, (int)u, true, {}, 0});
            accept_pending(v);
        }
    }
    for (uint64_t v = 0; v < n; ++v)
        if (peers[v].started) accept_pending(v);

    // ---- gossip ----
    std::unordered_map<std::string, int> index_of;  // hash -> message index
    uint64_t deliveries = 0, receipts = 0, sent_bytes = 0, recv_bytes = 0;
    auto broadcast = [&](int u, const std::string& line, Tracker& t) {  // peer.cpp:297-318
        for (size_t k = 0; k < peers[u].out.size(); ++k) {
            conns[peers[u].out[k]].buf += line;
            sent_bytes += line.size();
            if (t.sent_to.insert(peers[u].out_peer[k]).second) ++deliveries;
        }
    };
    for (uint32_t i = 0; i < n_msgs; ++i) {  // messageGenerationLoop (peer.cpp:357-379)
        const Gen& g = gen[i];
        if (g.origin >= n || !peers[g.origin].started) continue;
        Peer& p = peers[g.origin];
        const std::string content = gossip::message_content(p.addr);
        const std::string ts = gossip::message_timestamp(g.round);
        const std::string hash = gossip::message_hash(content, ts, p.addr.ip);
        if (index_of.count(hash)) die("two messages with one hash (same origin and round)");
        index_of[hash] = (int)i;
        Tracker& t = p.messages[hash];
        t.index = (int)i;
        broadcast((int)g.origin, gossip::gossip_json(content, hash, g.number, p.addr.ip, p.addr.port, ts) + "\n", t);
        p.log.push_back(gossip::peer_log_line(gossip::kEpochSeconds, "Generated message: " + content));
    }
    auto handle = [&](int v, const std::string& line) {  // handleClient (peer.cpp:255-295)
        std::string type, content, ts, ip, port, number, hash;
        if (!json_get(line, "type", &type) || type != "gossip" || !json_get(line, "content", &content) ||
            !json_get(line, "timestamp", &ts) || !json_get(line, "source_ip", &ip) ||
            !json_get(line, "source_port", &port) || !json_get(line, "msg_number", &number) ||
            !json_get(line, "hash", &hash)) {
            ++errors;
            return;
        }
        const std::string h = gossip::message_hash(content, ts, ip);  // calculateMessageHash, not the field
        if (h != hash || gossip::gossip_json(content, hash, std::atoi(number.c_str()), ip, std::atoi(port.c_str()),
                                             ts) != line.substr(0, line.size() - 1))
            ++errors;
        auto it = index_of.find(h);
        if (it == index_of.end()) {
            ++errors;
            return;
        }
        Peer& p = peers[v];
        if (p.messages.count(h)) return;  // duplicate: dropped
        Tracker& t = p.messages[h];
        t.index = it->second;
        ++receipts;
        p.log.push_back(gossip::peer_log_line(gossip::kEpochSeconds, "Received new message: " + content));
        broadcast(v, line, t);
    };
    std::vector<pollfd> pfd;
    while (true) {
        bool pending = false;
        pfd.clear();
        for (const Conn& c : conns) {
            pollfd x{c.fd, 0, 0};
            if (c.outgoing && c.off < c.buf.size()) {
                x.events = POLLOUT;
                pending = true;
            }
            if (!c.outgoing) x.events = POLLIN;
            pfd.push_back(x);
        }
        if (!pending && sent_bytes == recv_bytes) break;  // quiescent: nothing queued, nothing in flight
        if (poll(pfd.data(), pfd.size(), 5000) <= 0) die("poll (stalled)");
        for (size_t i = 0; i < conns.size(); ++i) {
            Conn& c = conns[i];
            if (c.outgoing && (pfd[i].revents & POLLOUT)) {
                const ssize_t k = write(c.fd, c.buf.data() + c.off, c.buf.size() - c.off);
                if (k < 0 && errno != EAGAIN) die("write");
                if (k > 0) c.off += (size_t)k;
                if (c.off == c.buf.size()) {
                    c.buf.clear();
                    c.off = 0;
                }
                errno = 0;
            } else if (!c.outgoing && (pfd[i].revents & (POLLIN | POLLHUP))) {
                char b[65536];
                const ssize_t k = read(c.fd, b, sizeof b);
                if (k < 0 && errno != EAGAIN) die("read");
                errno = 0;
                if (k <= 0) continue;
                recv_bytes += (uint64_t)k;
                c.buf.append(b, (size_t)k);
                size_t start = 0, nl;
                while ((nl = c.buf.find('\n', start)) != std::string::npos) {
                    handle(c.owner, c.buf.substr(start, nl + 1 - start));
                    start = nl + 1;
                }
                c.buf.erase(0, start);
            }
        }
    }
    for (const Conn& c : conns)
        if (!c.outgoing && !c.buf.empty()) ++errors;  // a partial message left over

    uint64_t started = 0;
    for (const Peer& p : peers) started += p.started;
    std::cout << "started " << started << "\n"
              << "deliveries " << deliveries << "\n"
              << "receipts " << receipts << "\n"
              << "refused " << refused << "\n"
              << "errors " << errors << "\n";
    for (uint64_t v = 0; v < n; ++v) {
        if (!peers[v].started) continue;
        std::vector<int> ids;
        for (const auto& kv : peers[v].messages) ids.push_back(kv.second.index);
        std::sort(ids.begin(), ids.end());
        std::cout << "seen " << v;
        for (int i : ids) std::cout << " " << i;
        std::cout << "\n";
        if (!log_dir.empty()) {
            std::ofstream f(log_dir + "/peer_" + std::to_string(peers[v].addr.port) + "_output.txt");
            for (const std::string& l : peers[v].log) f << l;
        }
    }
    for (const Conn& c : conns) close(c.fd);
    for (Peer& p : peers)
        if (p.listen_fd >= 0) close(p.listen_fd);
    for (int s = 0; s < n_seeds; ++s) {
        close(seed_fd[s]);
        delete seeds[s];
    }
    return 0;
}
