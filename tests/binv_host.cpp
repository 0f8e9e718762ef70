// Host harness for csrc/mbls_binv.hpp (the device inversion's algorithm, compiled here with g++):
// reads lines "<words> <hex word 0> ... <hex word words-1>" (12 = Fq modulus p, 8 = Fr modulus r),
// prints "<outer steps> <1 if the four-lane form (inverse_roles) agrees> <inverse words...>".  Driven by tests/test_oracle.py::test_binary_gcd_inverse.
#include <cstdio>
#include <cstdlib>

#include "mbls_binv.hpp"

static const uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                               0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
static const uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                              0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};

template <int N>
static void run(char* s, const uint32_t (&m)[N], uint32_t ninv) {
    uint32_t y[N], o[N];
    for (int i = 0; i < N; ++i) y[i] = (uint32_t)strtoul(s, &s, 16);
    const int steps = mbls::binv::inverse<N>(o, y, m, ninv);
    uint32_t q[N];
    const int qsteps = mbls::binv::inverse_roles<N>(q, y, m, ninv);  // the four-lane form, roles in turn
    bool same = qsteps == steps;
    for (int i = 0; i < N; ++i) same = same && q[i] == o[i];
    printf("%d %d", steps, same ? 1 : 0);
    for (int i = 0; i < N; ++i) printf(" %08x", o[i]);
    printf("\n");
}

int main() {
    char buf[1024];
    while (fgets(buf, sizeof buf, stdin)) {
        char* s = buf;
        const long words = strtol(s, &s, 10);
        if (words == 12)
            run<12>(s, P, 0xfffcfffdu);
        else
            run<8>(s, R, 0xffffffffu);
    }
    return 0;
}
