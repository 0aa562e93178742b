// TEST INFRASTRUCTURE: driver that links the reference's own, unmodified
// gpuraytrace/Graphics/Noise.cpp (compiled in place from /root/reference by
// oracle/Makefile) and dumps Noise::generate(false)'s tables (seed 300,
// Noise.cpp:39-94): linked as is, with this platform's CRT rand (glibc); linked with
// msvc_rand.cpp, with the MSVC CRT rand the reference's Windows build uses.  Used only
// to pin oracle/rt_oracle.c's and the product's table generators (tests/test_oracle.py,
// tests/test_host.py, fixtures by tests/golden/make_golden.py).
#include "Graphics/Noise.h"
#include <cstdio>

int main()
{
    Noise n;
    n.generate(false);
    std::fwrite(n.permutations2D, 1, Noise::TEXTURE_SIZE * Noise::TEXTURE_SIZE * 4, stdout);
    std::fwrite(n.permutations1D, sizeof(float), Noise::TEXTURE_SIZE * 4, stdout);
    return 0;
}
