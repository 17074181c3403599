// CPU check of nebula_amd/csrc/dtoa.h (the device's double -> string) against the oracle's rule:
// std::to_chars shortest digits formatted as Expression::toString (oracle/orc_expr.cpp).
// Usage: dtoa_check [count]  (exit 1 on the first mismatch)
#define NGX_DTOA_HOST
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "../nebula_amd/csrc/dtoa.h"

static std::string ref(double d) {                 // oracle/orc_expr.cpp Expression::toString
    if (std::isnan(d)) return "NaN";
    if (std::isinf(d)) return d < 0 ? "-Infinity" : "Infinity";
    if (d == 0) return std::signbit(d) ? "-0" : "0";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
    std::string sci(buf, r.ptr);
    bool neg = sci[0] == '-';
    if (neg) sci = sci.substr(1);
    auto epos = sci.find('e');
    int exp10 = std::atoi(sci.c_str() + epos + 1);
    std::string digits;
    for (size_t i = 0; i < epos; i++) if (sci[i] != '.') digits.push_back(sci[i]);
    int dp = exp10 + 1;
    std::string out = neg ? "-" : "";
    if (-6 < dp && dp <= 21) {
        if (dp <= 0) { out += "0."; out.append(static_cast<size_t>(-dp), '0'); out += digits; }
        else if (dp >= static_cast<int>(digits.size())) { out += digits; out.append(static_cast<size_t>(dp - static_cast<int>(digits.size())), '0'); }
        else { out += digits.substr(0, dp); out += "."; out += digits.substr(dp); }
    } else {
        out += digits.substr(0, 1);
        if (digits.size() > 1) { out += "."; out += digits.substr(1); }
        out += "E"; out += std::to_string(exp10);
    }
    return out;
}

static bool check(double d) {
    char out[64];
    const int n = ngx::dtoa::format(d, out);
    const std::string got(out, n), want = ref(d);
    if (got != want) {
        uint64_t b; std::memcpy(&b, &d, 8);
        std::printf("MISMATCH %016llx: got %s want %s\n", static_cast<unsigned long long>(b), got.c_str(), want.c_str());
        return false;
    }
    return true;
}

int main(int argc, char** argv) {
    const long count = argc > 1 ? std::atol(argv[1]) : 200000;
    std::mt19937_64 rng(12345);
    long n = 0;
    const double specials[] = {0.0, -0.0, 1.0, -1.0, 0.1, 0.2, 0.3, 1e21, 1e22, 1e-6, 1e-7, 123456789012345678.0,
                               5e-324, 2.2250738585072014e-308, 2.2250738585072009e-308, 1.7976931348623157e308,
                               9007199254740993.0, 3.14, 2.718281828459045, 1.0 / 3.0, 100.0, 1e15, 1e16, 1e17,
                               4.35, 0.000001, 0.0000001, 12345.6789, -9.87654321e-300, 1e308, 1e-308,
                               std::nan(""), INFINITY, -INFINITY};
    for (double d : specials) { if (!check(d)) return 1; n++; }
    for (int e = -1074; e <= 1023; e++) {                 // powers of two and their neighbours
        double p = std::ldexp(1.0, e);
        if (!check(p) || !check(std::nextafter(p, 0.0)) || !check(std::nextafter(p, INFINITY))) return 1;
        n += 3;
    }
    for (int e = -323; e <= 308; e++) {                   // powers of ten and their neighbours
        double p = std::pow(10.0, e);
        if (!std::isfinite(p) || p == 0) continue;
        if (!check(p) || !check(std::nextafter(p, 0.0)) || !check(std::nextafter(p, INFINITY))) return 1;
        n += 3;
    }
    for (long i = 0; i < count; i++) {
        uint64_t b = rng();
        double d;
        std::memcpy(&d, &b, 8);                            // every exponent, subnormals, NaNs
        if (!check(d)) return 1;
        double q = static_cast<double>(static_cast<int64_t>(rng() % 2000001) - 1000000) / static_cast<double>(1 + rng() % 10000);
        if (!check(q)) return 1;                           // "nice" decimals
        n += 2;
    }
    std::printf("OK %ld doubles\n", n);
    return 0;
}
