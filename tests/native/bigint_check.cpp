// Host build of csrc/nsg_bigint.h for tests/test_fraction_host.py: the same arithmetic the Fraction-coder
// kernel runs, exposed through a C ABI so the test can compare it with Python integers and fractions.Fraction.
// Test infrastructure only (built by the test with g++; never part of the product library).
#include "nsg_bigint.h"

using namespace nsg::bi;

extern "C" {

void bc_to_fraction(double p, uint64_t* num, int* shift, uint32_t* den) { to_fraction(p, num, shift, den); }

int bc_add(limb* o, const limb* a, int na, const limb* b, int nb) { return add(o, a, na, b, nb); }
int bc_sub(limb* o, const limb* a, int na, const limb* b, int nb) { return sub(o, a, na, b, nb); }
int bc_mul(limb* o, const limb* a, int na, const limb* b, int nb) { return mul(o, a, na, b, nb); }
int bc_mul_u64(limb* o, const limb* a, int na, uint64_t m) { return mul_u64(o, a, na, m); }
int bc_shl(limb* o, const limb* a, int na, int k) { return shl(o, a, na, k); }
int bc_shr(limb* o, const limb* a, int na, int k) { return shr(o, a, na, k); }
uint32_t bc_divmod_u32(limb* q, const limb* a, int na, uint32_t d) { return divmod_u32(q, a, na, d); }
int bc_divmod(limb* q, limb* r, int* nr, const limb* u, int m, const limb* v, int n, limb* un, limb* vn) {
    return divmod(q, r, nr, u, m, v, n, un, vn);
}
int bc_cmp(const limb* a, int na, const limb* b, int nb) { return cmp(a, na, b, nb); }
}
