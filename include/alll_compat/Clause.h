// Clause.h -- compatibility header (API of the reference's library/include/Clause.h:17-46).
#ifndef ALLL_COMPAT_CLAUSE_H
#define ALLL_COMPAT_CLAUSE_H

#include <vector>

#include "VariablesArray.h"

template <typename tV>
class Clause {
   public:
    typedef std::vector<Clause<tV>*> ClauseArray;

    std::vector<tV>* literals;
    unsigned short int t_id{};

    explicit Clause(std::vector<tV>* lits, unsigned short int tid) : literals(lits), t_id(tid) {}

    // true iff no literal is true; literal l is true iff vars[l >> 1] XOR (l & 1)
    bool is_not_satisfied(const bool* vars) const {
        for (const tV l : *literals)
            if (vars[l >> 1] != static_cast<bool>(l & 1)) return false;
        return true;
    }
};

#endif
