// Host-side planner for the LDS Stockham FFT (fft_lds.h).
#pragma once

#include <vector>

#include "fft_lds.h"

namespace gsdr
{
namespace fft
{

// Radices the device code implements, largest first.
static const int kRadices[] = {25, 20, 16, 12, 10, 8, 6, 5, 4, 3, 2};

// Fits: every butterfly of the stage must be owned by a thread (bpt_for(R) each).
inline bool stage_fits(int n, int R, int nt) { return n / R <= nt * bpt_for(R); }

inline bool search(int n, int rem, int nt, int depth_left, std::vector<int>& cur, std::vector<int>& best)
{
    if (rem == 1)
        {
            if (best.empty() || cur.size() < best.size()) best = cur;
            return true;
        }
    if (depth_left == 0) return false;
    if (!best.empty() && (int)cur.size() + 1 >= (int)best.size()) return false;
    bool found = false;
    for (int R : kRadices)
        {
            if (rem % R != 0 || !stage_fits(n, R, nt)) continue;
            cur.push_back(R);
            found |= search(n, rem / R, nt, depth_left - 1, cur, best);
            cur.pop_back();
        }
    return found;
}

// Minimum-stage factorisation of n for an nt-thread workgroup; false if n has a
// prime factor outside {2,3,5} or no plan satisfies the per-thread budget.
inline bool make_plan(int n, int nt, Plan& plan)
{
    if (n < 2) return false;
    std::vector<int> cur, best;
    search(n, n, nt, kMaxStages, cur, best);
    if (best.empty()) return false;
    plan.n = n;
    plan.nstages = (int)best.size();
    for (int i = 0; i < kMaxStages; ++i) plan.radix[i] = i < plan.nstages ? best[i] : 1;
    return true;
}

}  // namespace fft
}  // namespace gsdr
