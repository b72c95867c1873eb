// ClauseGenerator.h -- compatibility header (API of the reference's
// library/include/ClauseGenerator.h:12-114): a host-side enumerator over a clause callback.
// The GPU streaming solve does not use it (SATInstance::solve(getEnumeratedClause, ...)
// materialises the instance once and reproduces this generator's yield order on the device);
// it is kept for code that drives a generator directly.
//
// Behaviour restated from the reference: clauses are enumerated by index within
// [base_offset, base_offset + n_clauses); yieldRandomUNSATClauseBatch visits batch_size steps
// of the walk c <- (c + P) % n_clauses (P = 9223372036854775783, c kept across calls and resets)
// and returns the clauses the assignment violates; yieldNextClause walks indices in order;
// both reset once every clause has been yielded.
#ifndef ALLL_COMPAT_CLAUSEGENERATOR_H
#define ALLL_COMPAT_CLAUSEGENERATOR_H

#include <cstdint>
#include <iostream>
#include <type_traits>

#include "Clause.h"

template <class T, class Enable = void>
class ClauseGenerator {};

template <class T>
class ClauseGenerator<T, typename std::enable_if<std::is_integral<T>::value>::type> {
   public:
    using ClauseArray = typename Clause<T>::ClauseArray;
    typedef unsigned short int t_id_T;

    T n_clauses;

    ClauseGenerator(Clause<T>* (*getEnumeratedClause)(T, t_id_T), t_id_T t_id, T n_clauses, T base_offset,
                    T batch_size)
        : n_clauses(n_clauses), get_(getEnumeratedClause), batch_(batch_size), base_(base_offset), t_id_(t_id) {}

    ClauseArray* yieldRandomUNSATClauseBatch(const bool* var_arr) {
        if (finished_) reset();
        auto out = new ClauseArray();
        const T n = (yielded_ + batch_ >= n_clauses) ? n_clauses - yielded_ : batch_;
        for (T i = 0; i < n; i++) {
            walk_ = (walk_ + kStep) % n_clauses;
            Clause<T>* cl = get_(base_ + walk_, t_id_);
            if (cl == nullptr) {
                std::cerr << "WARNING: Clause generator went out of range and yielded nullptr." << std::endl;
                finished_ = true;
                break;
            }
            if (cl->is_not_satisfied(var_arr)) {
                out->push_back(cl);
            } else {
                delete cl->literals;
                delete cl;
            }
            yielded_++;
        }
        if (yielded_ == n_clauses) finished_ = true;
        return out;
    }

    Clause<T>* yieldNextClause() {
        if (finished_) reset();
        Clause<T>* cl = get_(base_ + yielded_, t_id_);
        if (cl == nullptr) {
            std::cerr << "WARNING: Clause generator went out of range and yielded nullptr." << std::endl;
            finished_ = true;
            return nullptr;
        }
        if (++yielded_ == n_clauses) finished_ = true;
        return cl;
    }

    bool has_finished_yielding() { return finished_; }

    void reset() {
        yielded_ = 0;
        finished_ = false;
    }

   private:
    static constexpr uint64_t kStep = 9223372036854775783ull;
    Clause<T>* (*get_)(T, unsigned short int);
    T batch_, base_;
    t_id_T t_id_{};
    T walk_ = 0;
    bool finished_ = false;
    T yielded_ = 0;
};

#endif
