// VariablesArray.h -- compatibility header (API of the reference's
// library/include/VariablesArray.h:17-35).  The initial values are the solver's seeded
// Philox initial assignment (seed: env ALLL_SEED, default 1) instead of std::random_device, or with
// env ALLL_REFERENCE_RNG=<state> the reference's own fill from the random_device stand-in.
#ifndef ALLL_COMPAT_VARIABLESARRAY_H
#define ALLL_COMPAT_VARIABLESARRAY_H

#include <cstdint>
#include <cstdlib>

#include "RandomBoolGenerator.h"
#include "alll.h"

namespace alll_compat {
inline uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* s = std::getenv(name);
    return (s && *s) ? std::strtoull(s, nullptr, 10) : dflt;
}
}  // namespace alll_compat

template <typename tV>
class VariablesArray {
   public:
    tV n_vars;
    bool* vars;

    explicit VariablesArray(tV n) : n_vars(n), vars(new bool[n > 0 ? n : 1]) {
        uint8_t* tmp = new uint8_t[n > 0 ? n : 1];
        // ALLL_REFERENCE_RNG=<state>: the reference's own fill from the random_device stand-in
        // (DESIGN.md §1.1); else the solver's Philox fill
        if (std::getenv("ALLL_REFERENCE_RNG") && *std::getenv("ALLL_REFERENCE_RNG"))
            alll_reference_initial_assignment(alll_compat::env_u64("ALLL_REFERENCE_RNG", 0), (uint32_t)n, tmp);
        else
            alll_initial_assignment(alll_compat::env_u64("ALLL_SEED", 1), (uint32_t)n, tmp);
        for (tV i = 0; i < n; ++i) vars[i] = tmp[i] != 0;
        delete[] tmp;
    }
};

#endif
