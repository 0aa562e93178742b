// TEST INFRASTRUCTURE: the MSVC CRT rand()/srand() (x = x * 214013 + 2531011, rand = (x >> 16) &
// 0x7fff; state seeded by srand, initial state 1), linked INTO oracle/_ref/ref_noise_dump_msvc so
// that the reference's unmodified Graphics/Noise.cpp (Noise::generate, Noise.cpp:39-56: srand(300),
// swap(p[x], p[rand() % 128])) resolves rand/srand to these definitions instead of glibc's: the
// executable's own symbols take precedence over libc's.  This reproduces the tables the reference
// builds on its platform (Windows, vcredist CRT).
static unsigned int g_state = 1u;

extern "C" void srand(unsigned int seed) { g_state = seed; }

extern "C" int rand(void)
{
    g_state = g_state * 214013u + 2531011u;
    return (int)((g_state >> 16) & 0x7fffu);
}
