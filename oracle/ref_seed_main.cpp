// ref_seed_main.cpp -- TEST INFRASTRUCTURE ONLY.
// The reference ships no seed program; this main runs the reference's own SeedNode
// (seed.cpp:15-204, compiled where it lies under /root/reference by oracle/Makefile, output to oracle/_ref/)
// as a TCP seed on 127.0.0.1:<port>, logging to seed_<port>_output.txt in the working directory.  Used only by
// tests/golden/make_ref_wire_golden.py, which records the reference's wire bytes and logs as fixtures.
#include "seed.hpp"
#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: %s <port>\n", argv[0]);
        return 2;
    }
    SeedNode seed("127.0.0.1", std::atoi(argv[1]));
    return seed.start() ? 0 : 1;
}
