// RowWriter (src/dataman/RowWriter.{h,cpp,inl}) restated for rows of a response schema (version 0,
// so no version bytes): header byte = offset bytes - 1, then one block offset per 16 fields, then the
// field data ("cord"). A value goes through RowWriter::operator<< of its value type into the field type
// of the column it lands in, as PropsCollector writes it (src/storage/Collector.h:38-84). Shared by
// the device row encoder (kernels.hip k_encode_rows) and the host TagData rows (engine.cpp).
#pragma once

#include "ngx_device.h"

namespace ngx {

struct RowSink {
    uint8_t* p;                         // nullptr: count only
    uint64_t n;
    __host__ __device__ inline void put(uint8_t b) { if (p) p[n] = b; n++; }
    __host__ __device__ inline void le(uint64_t v, int bytes) {
        for (int k = 0; k < bytes; k++) put(static_cast<uint8_t>(v >> (8 * k)));
    }
    __host__ __device__ inline void varint(uint64_t v) {                  // folly::encodeVarint (LEB128)
        while (v >= 0x80) { put(static_cast<uint8_t>(v | 0x80)); v >>= 7; }
        put(static_cast<uint8_t>(v));
    }
};

// value of VM type vt (V_INT / V_DBL / V_BOOL / V_STR; x = int, double bits, bool, or a pointer to
// len string bytes) into a field of SupportedType ft
__host__ __device__ inline void rowField(RowSink& s, uint8_t vt, int64_t x, uint32_t len, int32_t ft) {
    switch (vt) {
        case V_INT:                                      // integral operator<<, RowWriter.inl:9-34
            if (ft == 2 || ft == 21) s.varint(static_cast<uint64_t>(x));
            else if (ft == 3) s.le(static_cast<uint64_t>(x), 8);
            else s.varint(0);
            break;
        case V_BOOL: s.put(ft == 1 && x != 0 ? 1 : 0); break;                // RowWriter.cpp:98-114
        case V_DBL:                                      // RowWriter.cpp:139-157
            if (ft == 4) s.le(__builtin_bit_cast(uint32_t, static_cast<float>(__builtin_bit_cast(double, x))), 4);
            else s.le(ft == 5 ? static_cast<uint64_t>(x) : 0ULL, 8);
            break;
        case V_STR:                                      // RowWriter.cpp:164-182
            if (ft == 6) {
                s.varint(len);
                const uint8_t* b = reinterpret_cast<const uint8_t*>(x);
                for (uint32_t k = 0; k < len; k++) s.put(b[k]);
            } else {
                s.varint(0);
            }
            break;
        default: break;
    }
}

// operator<<(Skip) default of a field never written (RowWriter.cpp:213-263)
__host__ __device__ inline void rowDefault(RowSink& s, int32_t ft) {
    switch (ft) {
        case 1: s.put(0); break;
        case 4: s.le(0, 4); break;
        case 5: case 3: s.le(0, 8); break;
        default: s.varint(0); break;                     // INT / TIMESTAMP / STRING
    }
}

// calcOccupiedBytes (RowWriter.cpp:90-98)
__host__ __device__ inline int rowOffsetBytes(uint64_t v) {
    int b = 1;
    for (v >>= 8; v; v >>= 8) b++;
    return b;
}

}  // namespace ngx
