// poa_identity.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/liboracle.so).
//
// Banded Levenshtein distance for the accuracy sanity check of SURVEY.md
// §4-5: the CCS of a synthetic ZMW against the generator's true insert.  Not
// part of the reference's algorithm; not parity.  The band (diagonals
// j - i within `band` of the straight path, widened by the length
// difference) makes the result an upper bound of the edit distance, so the
// identity it gives is a lower bound -- conservative for the check.
#include <stdint.h>
#include <stdlib.h>

int64_t ocsx_edit_distance(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb, uint32_t band)
{
    const int64_t dl = (int64_t)lb - (int64_t)la;
    const int64_t lo = -(int64_t)band + (dl < 0 ? dl : 0), hi = (int64_t)band + (dl > 0 ? dl : 0);
    const int64_t w = hi - lo + 1, inf = (int64_t)1 << 40;
    int64_t *prev = malloc(sizeof(int64_t) * (size_t)(w + 2)), *cur = malloc(sizeof(int64_t) * (size_t)(w + 2));
    if (!prev || !cur) {
        free(prev);
        free(cur);
        return -1;
    }
    // slot k + 1 holds diagonal d = lo + k; slots 0 and w + 1 stay inf
    for (int64_t k = 0; k < w + 2; ++k) prev[k] = cur[k] = inf;
    for (int64_t d = lo; d <= hi; ++d)
        if (d >= 0 && d <= (int64_t)lb) prev[d - lo + 1] = d;  // row 0: D[0][j] = j
    for (int64_t i = 1; i <= (int64_t)la; ++i) {
        for (int64_t d = lo; d <= hi; ++d) {
            const int64_t j = i + d, k = d - lo + 1;
            if (j < 0 || j > (int64_t)lb) {
                cur[k] = inf;
                continue;
            }
            int64_t v = j == 0 ? i : inf;
            if (j >= 1) {
                const int64_t s = prev[k] + (a[i - 1] != b[j - 1]);  // D[i-1][j-1]
                if (s < v) v = s;
                if (cur[k - 1] + 1 < v) v = cur[k - 1] + 1;  // D[i][j-1]
            }
            if (prev[k + 1] + 1 < v) v = prev[k + 1] + 1;  // D[i-1][j]
            cur[k] = v;
        }
        int64_t *t = prev;
        prev = cur;
        cur = t;
    }
    const int64_t r = prev[dl - lo + 1];
    free(prev);
    free(cur);
    return r >= inf ? -1 : r;
}
