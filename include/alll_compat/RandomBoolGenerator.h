// RandomBoolGenerator.h -- compatibility header (API of the reference's
// library/include/RandomBoolGenerator.h:14-50).  The device solver does not use it: its
// resampling is Philox4x32-10 keyed by (seed, iteration, variable).  Kept so code that
// names RBG<E> / ull keeps compiling.
#ifndef ALLL_COMPAT_RANDOMBOOLGENERATOR_H
#define ALLL_COMPAT_RANDOMBOOLGENERATOR_H

#include <random>

typedef unsigned long long ull;

template <typename E>
class RBG {
   public:
    explicit RBG(E& engine) : engine_(engine) {}

    // One bit per call, drawn 32 at a time from a 32-bit uniform draw.
    bool sample() {
        if (left_ == 0) {
            bits_ = std::uniform_int_distribution<unsigned int>{}(engine_);
            left_ = 32;
        }
        const bool b = bits_ & 1u;
        bits_ >>= 1;
        --left_;
        return b;
    }

   private:
    E engine_;
    unsigned int bits_ = 0;
    int left_ = 0;
};

#endif
