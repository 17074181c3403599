// Shortest round-trip decimal of a double — the digits double-conversion's SHORTEST mode and
// std::to_chars produce — for `(string)` casts on the device (Expression::toString of a double,
// restated in oracle/orc_expr.cpp). Exact integer arithmetic (Burger & Dybvig's free-format
// algorithm, "Printing Floating-Point Numbers Quickly and Accurately", PLDI '96): the value and the
// halfway points to its neighbours as ratios of ~1100-bit integers; digits are generated until the
// remainder falls inside the rounding interval (inclusive when the significand is even: a decimal on
// the boundary parses back to it under round-half-even). No tables, no floating point; slow next to
// table-driven printers, but it runs only for the rare double-to-string cast.
//
// Compiled for the device (vm.h) and, for the CPU test against std::to_chars, for the host
// (tests/dtoa_check.cpp with NGX_DTOA_HOST).
#pragma once

#ifdef NGX_DTOA_HOST
#include <cstdint>
#define NGX_DTOA_FN static inline
#else
#define NGX_DTOA_FN static __device__ __noinline__
#endif

namespace ngx {
namespace dtoa {

constexpr int kLimbs = 38;                     // 1216 bits: 2^1075 scaled by up to 10^2, with headroom

struct Big {
    uint32_t w[kLimbs];
    int n;                                     // limbs in use (w[n - 1] != 0, or n == 0)
};

NGX_DTOA_FN void setU64(Big& a, uint64_t v) {
    a.n = 0;
    for (int i = 0; i < kLimbs; i++) a.w[i] = 0;
    while (v) { a.w[a.n++] = static_cast<uint32_t>(v); v >>= 32; }
}
NGX_DTOA_FN void mulSmall(Big& a, uint32_t m) {
    uint64_t carry = 0;
    for (int i = 0; i < a.n; i++) {
        const uint64_t t = static_cast<uint64_t>(a.w[i]) * m + carry;
        a.w[i] = static_cast<uint32_t>(t);
        carry = t >> 32;
    }
    if (carry && a.n < kLimbs) a.w[a.n++] = static_cast<uint32_t>(carry);
}
NGX_DTOA_FN void shl(Big& a, int bits) {
    if (a.n == 0 || bits == 0) return;
    const int words = bits / 32, b = bits % 32;
    int n = a.n + words + 1;
    if (n > kLimbs) n = kLimbs;
    for (int i = n - 1; i >= 0; i--) {
        const int src = i - words;
        uint32_t hi = src >= 0 && src < a.n ? a.w[src] : 0u;
        uint32_t lo = src - 1 >= 0 && src - 1 < a.n ? a.w[src - 1] : 0u;
        a.w[i] = b ? (hi << b) | (lo >> (32 - b)) : hi;
    }
    a.n = n;
    while (a.n > 0 && a.w[a.n - 1] == 0) a.n--;
}
NGX_DTOA_FN int cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int i = a.n - 1; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}
// a + b compared with c, without forming the sum in place
NGX_DTOA_FN int cmpSum(const Big& a, const Big& b, const Big& c) {
    Big t;
    t.n = a.n > b.n ? a.n : b.n;
    uint64_t carry = 0;
    for (int i = 0; i < kLimbs; i++) {
        const uint64_t s = static_cast<uint64_t>(i < a.n ? a.w[i] : 0u) + (i < b.n ? b.w[i] : 0u) + carry;
        t.w[i] = static_cast<uint32_t>(s);
        carry = s >> 32;
    }
    while (t.n < kLimbs && t.w[t.n] != 0) t.n++;             // the carry out of the top limb
    while (t.n > 0 && t.w[t.n - 1] == 0) t.n--;
    return cmp(t, c);
}
NGX_DTOA_FN void sub(Big& a, const Big& b) {     // a -= b, a >= b
    int64_t borrow = 0;
    for (int i = 0; i < a.n; i++) {
        int64_t d = static_cast<int64_t>(a.w[i]) - (i < b.n ? b.w[i] : 0u) - borrow;
        borrow = d < 0;
        a.w[i] = static_cast<uint32_t>(d + (borrow << 32));
    }
    while (a.n > 0 && a.w[a.n - 1] == 0) a.n--;
}
NGX_DTOA_FN void mulPow10(Big& a, int k) {
    for (; k >= 9; k -= 9) mulSmall(a, 1000000000u);
    uint32_t p = 1;
    for (; k > 0; k--) p *= 10u;
    if (p > 1) mulSmall(a, p);
}

// digits of |v| (v finite, nonzero) into dig[], count returned; v = 0.d1 d2 ... x 10^k
NGX_DTOA_FN int shortest(double v, char* dig, int& k) {
    uint64_t bits;
    __builtin_memcpy(&bits, &v, 8);
    const int be = static_cast<int>((bits >> 52) & 0x7FF);
    uint64_t f = bits & ((1ULL << 52) - 1);
    int e;
    if (be == 0) { e = -1074; } else { f |= 1ULL << 52; e = be - 1075; }
    const bool even = (f & 1) == 0;
    // v = r / s; the rounding interval is (v - mm / s, v + mp / s)
    Big r, s, mp, mm;
    const bool lowerCloser = be > 1 && f == (1ULL << 52);   // the neighbour below is half as far
    if (e >= 0) {
        setU64(r, f); shl(r, e + 1 + (lowerCloser ? 1 : 0));
        setU64(s, lowerCloser ? 4 : 2);
        setU64(mp, 1); shl(mp, e + (lowerCloser ? 1 : 0));
        setU64(mm, 1); shl(mm, e);
    } else {
        setU64(r, f); shl(r, lowerCloser ? 2 : 1);
        setU64(s, 1); shl(s, -e + (lowerCloser ? 2 : 1));
        setU64(mp, lowerCloser ? 2 : 1);
        setU64(mm, 1);
    }
    // k ~ ceil(log10 v): log10(2) * (e + bit length of f), corrected below
    int bl = 0;
    for (uint64_t t = f; t; t >>= 1) bl++;
    k = static_cast<int>((static_cast<int64_t>(e + bl) * 78913 + (1 << 18) - 1) >> 18);   // 78913 / 2^18 ~ log10 2
    if (k >= 0) mulPow10(s, k);
    else { mulPow10(r, -k); mulPow10(mp, -k); mulPow10(mm, -k); }
    // fixup: high end of the interval must lie below s (s * 10^-k is the first digit's unit)
    while (true) {
        const int c = cmpSum(r, mp, s);
        if (even ? c >= 0 : c > 0) { mulSmall(s, 10); k++; } else break;
    }
    while (true) {
        Big r10 = r, mp10 = mp;
        mulSmall(r10, 10); mulSmall(mp10, 10);
        const int c = cmpSum(r10, mp10, s);
        if (even ? c < 0 : c <= 0) { r = r10; mp = mp10; mulSmall(mm, 10); k--; } else break;
    }
    int n = 0;
    while (n < 24) {
        mulSmall(r, 10); mulSmall(mp, 10); mulSmall(mm, 10);
        int d = 0;
        while (cmp(r, s) >= 0) { sub(r, s); d++; }
        const int cl = cmp(r, mm), ch = cmpSum(r, mp, s);
        const bool low = even ? cl <= 0 : cl < 0;
        const bool high = even ? ch >= 0 : ch > 0;
        if (!low && !high) { dig[n++] = static_cast<char>('0' + d); continue; }
        if (low && !high) { dig[n++] = static_cast<char>('0' + d); break; }
        if (high && !low) { dig[n++] = static_cast<char>('0' + d + 1); break; }
        // both ends reachable: the closer digit, a tie to the even one
        Big r2 = r;
        mulSmall(r2, 2);
        const int c2 = cmp(r2, s);
        dig[n++] = static_cast<char>('0' + ((c2 < 0 || (c2 == 0 && d % 2 == 0)) ? d : d + 1));
        break;
    }
    return n;
}

// Expression::toString of a double (orc_expr.cpp): NaN, [-]Infinity, [-]0, else the shortest digits,
// plain when -6 < decimal point <= 21, else d[.ddd]E<exp>. Returns the length written to out (<= 32).
NGX_DTOA_FN int format(double v, char* out) {
    uint64_t bits;
    __builtin_memcpy(&bits, &v, 8);
    const bool neg = bits >> 63;
    int n = 0;
    auto put = [&](const char* s) { while (*s) out[n++] = *s++; };
    if (((bits >> 52) & 0x7FF) == 0x7FF) {
        if (bits & ((1ULL << 52) - 1)) { put("NaN"); return n; }
        put(neg ? "-Infinity" : "Infinity");
        return n;
    }
    if (neg) out[n++] = '-';
    if ((bits << 1) == 0) { out[n++] = '0'; return n; }
    char dig[24];
    int k = 0;
    const int nd = shortest(neg ? -v : v, dig, k);
    const int dp = k;                              // the decimal point after dp digits
    if (-6 < dp && dp <= 21) {
        if (dp <= 0) {
            out[n++] = '0'; out[n++] = '.';
            for (int i = 0; i < -dp; i++) out[n++] = '0';
            for (int i = 0; i < nd; i++) out[n++] = dig[i];
        } else if (dp >= nd) {
            for (int i = 0; i < nd; i++) out[n++] = dig[i];
            for (int i = nd; i < dp; i++) out[n++] = '0';
        } else {
            for (int i = 0; i < dp; i++) out[n++] = dig[i];
            out[n++] = '.';
            for (int i = dp; i < nd; i++) out[n++] = dig[i];
        }
    } else {
        out[n++] = dig[0];
        if (nd > 1) { out[n++] = '.'; for (int i = 1; i < nd; i++) out[n++] = dig[i]; }
        out[n++] = 'E';
        int x = dp - 1;
        if (x < 0) { out[n++] = '-'; x = -x; }
        char t[4];
        int m = 0;
        do { t[m++] = static_cast<char>('0' + x % 10); x /= 10; } while (x);
        while (m) out[n++] = t[--m];
    }
    return n;
}

}  // namespace dtoa
}  // namespace ngx
