// tv_core.h -- the binary Tal-Vardy core shared by the binary (tv_construct.cpp) and q-ary
// (qary_construct.cpp) constructions: letters, the reference's merge / degrade / upgrade with
// the bookkeeping of which input letters went where (the reference's `auxiliary` lists).
#pragma once
#include <stdint.h>

#include <vector>

namespace pcub {
namespace tv {

struct Letter {
    double p0, p1;
};

// Failures the reference reports as Python exceptions (PCUB_E* codes of polarcub_construct.h).
struct Err {
    int code = 0;
    void set(int c) {
        if (!code) code = c;
    }
};

// upgrade auxiliary of one output letter: merged-letter indices in its [left, centre, right]
// sets (BinaryMemorylessDistribution.upgrade, ScalarDistributions/BinaryMemorylessDistribution.py:360)
struct UpAux {
    std::vector<int64_t> l, c, r;
};

double py_sum(const Letter& l);
double eta(double p, Err& err);
bool py_isclose(double a, double b);
// mergeEquivalentSymbols (:167-208); grp[k] = merged letter of input letter k, -1 = dropped
void merge_equivalent(std::vector<Letter>& p, std::vector<int64_t>* grp, Err& err);
// degrade(L) (:287-346) on merged letters; grp[k] = output letter of merged letter k
std::vector<Letter> degrade_merged(const std::vector<Letter>& in, int64_t L, std::vector<int64_t>* grp, Err& err);
// upgrade(L) (:348-427) on merged letters; aux (optional) per output letter
std::vector<Letter> upgrade_merged(const std::vector<Letter>& in, int64_t L, Err& err, std::vector<UpAux>* aux);

}  // namespace tv
}  // namespace pcub
