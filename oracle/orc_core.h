// =====================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.
//
//  A plain C++ CPU restatement of the reference (NebulaGraph v1.x, /root/reference) storage
//  GetNeighbors path and the graphd GoExecutor, used as the parity checker for the
//  MI355X product in nebula_amd/. Only tests/, __graft_entry__.smoke() and bench.py's
//  cpu_baseline leg may load it. Nothing under nebula_amd/ links, includes or calls it.
//
//  Pinning: the restatement is checked against the reference's own known answers
//  (QueryBoundTest, GoTest on the NBA fixture, ExpressionTest, RowReaderTest/RowWriterTest,
//  NebulaKeyUtilsTest) in tests/test_oracle_*.py. The reference itself cannot be built or run
//  in this pipeline, so those fixtures are the pin.
//
//  This header: ids/types, Status, the key codec (NebulaKeyUtils), schemas, RowReader and
//  RowWriter (dataman).
// =====================================================================================
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <variant>
#include <vector>

namespace orc {

using VertexID = int64_t;     // src/common/base/ThriftTypes.h:15-30
using EdgeType = int32_t;
using TagID = int32_t;
using PartitionID = int32_t;
using EdgeRanking = int64_t;
using SchemaVer = int64_t;
using GraphSpaceID = int32_t;

// src/interface/common.thrift:30-56
enum SupportedType : int32_t {
    UNKNOWN = 0, BOOL = 1, INT = 2, VID = 3, FLOAT = 4, DOUBLE = 5, STRING = 6, TIMESTAMP = 21,
};

// VariantType = boost::variant<int64_t, double, bool, std::string>   (src/common/base/Base.h:140)
using Variant = std::variant<int64_t, double, bool, std::string>;
enum { VAR_INT64 = 0, VAR_DOUBLE = 1, VAR_BOOL = 2, VAR_STR = 3 };

// Minimal Status / StatusOr (src/common/base/Status.h) — only ok() and a message matter here.
struct Status {
    bool ok_ = true;
    std::string msg_;
    static Status OK() { return Status(); }
    static Status Error(std::string m) { Status s; s.ok_ = false; s.msg_ = std::move(m); return s; }
    bool ok() const { return ok_; }
};

template <typename T>
struct StatusOr {
    Status status_;
    T value_{};
    StatusOr() : status_(Status::Error("uninitialized")) {}
    StatusOr(Status s) : status_(std::move(s)) {}                 // NOLINT
    StatusOr(T v) : value_(std::move(v)) {}                        // NOLINT
    bool ok() const { return status_.ok(); }
    const T& value() const { return value_; }
    T& value() { return value_; }
    const Status& status() const { return status_; }
};

// OptVariantType (src/common/filter/Expressions.h:20). A few constructors for convenience so that
// returning an int64/double/bool/string directly builds the variant, as boost does there.
struct OptVariant : StatusOr<Variant> {
    OptVariant() = default;
    OptVariant(Status s) : StatusOr<Variant>(std::move(s)) {}     // NOLINT
    OptVariant(Variant v) : StatusOr<Variant>(std::move(v)) {}    // NOLINT
    OptVariant(int64_t v) : StatusOr<Variant>(Variant(v)) {}      // NOLINT
    OptVariant(double v) : StatusOr<Variant>(Variant(v)) {}       // NOLINT
    OptVariant(bool v) : StatusOr<Variant>(Variant(v)) {}         // NOLINT
    OptVariant(std::string v) : StatusOr<Variant>(Variant(std::move(v))) {}  // NOLINT
};

inline int which(const Variant& v) { return static_cast<int>(v.index()); }

// ID_HASH (src/common/base/Base.h:166-167)
inline PartitionID idHash(int64_t id, int64_t numShards) {
    return static_cast<PartitionID>(static_cast<uint64_t>(id) % static_cast<uint64_t>(numShards) + 1);
}

// -------------------------------------------------------------------------------------
//  Key codec — restates src/common/utils/NebulaKeyUtils.{h,cpp}
//  vertex: item(4) vid(8) tag(4) version(8) = 24 bytes
//  edge:   item(4) src(8) type(4) rank(8) dst(8) version(8) = 40 bytes
//  item = (part << 8) | kData(1); edge type stored as type | 0x40000000 (NebulaKeyUtils.cpp:33)
// -------------------------------------------------------------------------------------
namespace keys {
constexpr int32_t kVertexLen = 24;
constexpr int32_t kEdgeLen = 40;
constexpr uint32_t kTypeMask = 0x000000FF;
constexpr uint32_t kTagEdgeMask = 0x40000000;
constexpr uint32_t kData = 1;

template <typename T>
inline T readInt(const char* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }
template <typename T>
inline void app(std::string& s, T v) { s.append(reinterpret_cast<const char*>(&v), sizeof(T)); }

inline std::string edgeKey(PartitionID part, VertexID src, EdgeType type, EdgeRanking rank,
                           VertexID dst, int64_t ver) {          // NebulaKeyUtils.cpp:27-45
    type = static_cast<EdgeType>(static_cast<uint32_t>(type) | kTagEdgeMask);
    int32_t item = (part << 8) | static_cast<int32_t>(kData);
    std::string k; k.reserve(kEdgeLen);
    app(k, item); app(k, src); app(k, type); app(k, rank); app(k, dst); app(k, ver);
    return k;
}
inline std::string vertexKey(PartitionID part, VertexID vid, TagID tag, int64_t ver) {  // :12-24
    tag = static_cast<TagID>(static_cast<uint32_t>(tag) & ~kTagEdgeMask);
    int32_t item = (part << 8) | static_cast<int32_t>(kData);
    std::string k; k.reserve(kVertexLen);
    app(k, item); app(k, vid); app(k, tag); app(k, ver);
    return k;
}
inline std::string edgePrefix(PartitionID part, VertexID src, EdgeType type) {  // :156-166
    type = static_cast<EdgeType>(static_cast<uint32_t>(type) | kTagEdgeMask);
    int32_t item = (part << 8) | static_cast<int32_t>(kData);
    std::string k; app(k, item); app(k, src); app(k, type);
    return k;
}
inline std::string vertexPrefix(PartitionID part, VertexID vid, TagID tag) {  // :143-153
    tag = static_cast<TagID>(static_cast<uint32_t>(tag) & ~kTagEdgeMask);
    int32_t item = (part << 8) | static_cast<int32_t>(kData);
    std::string k; app(k, item); app(k, vid); app(k, tag);
    return k;
}
inline PartitionID getPart(const char* k) { return readInt<int32_t>(k) >> 8; }   // .h:116-118
inline bool isEdge(const char* k, size_t n) {                                      // .h:155-167
    if (n != kEdgeLen) return false;
    if ((readInt<uint32_t>(k) & kTypeMask) != kData) return false;
    return (readInt<int32_t>(k + 12) & static_cast<int32_t>(kTagEdgeMask)) != 0;
}
inline bool isVertex(const char* k, size_t n) {                                    // .h:120-132
    if (n != kVertexLen) return false;
    if ((readInt<uint32_t>(k) & kTypeMask) != kData) return false;
    return (readInt<int32_t>(k + 12) & static_cast<int32_t>(kTagEdgeMask)) == 0;
}
inline VertexID getSrcId(const char* k) { return readInt<int64_t>(k + 4); }        // .h:189-192
inline VertexID getDstId(const char* k) { return readInt<int64_t>(k + 24); }       // .h:194-199
inline EdgeType getEdgeType(const char* k) {                                       // .h:201-206
    EdgeType t = readInt<int32_t>(k + 12);
    return t > 0 ? static_cast<EdgeType>(static_cast<uint32_t>(t) & ~kTagEdgeMask) : t;
}
inline EdgeRanking getRank(const char* k) { return readInt<int64_t>(k + 16); }     // .h:208-212
inline VertexID getVertexId(const char* k) { return readInt<int64_t>(k + 4); }
inline TagID getTagId(const char* k) { return readInt<int32_t>(k + 12); }
}  // namespace keys

// -------------------------------------------------------------------------------------
//  Schemas — the parts of SchemaProviderIf / NebulaSchemaProvider / ResultSchemaProvider used
//  by the path: field lookup by name/index (unknown => UNKNOWN type / -1), version, TTL.
// -------------------------------------------------------------------------------------
struct Field {
    std::string name;
    SupportedType type;
};

struct Schema {
    SchemaVer ver = 0;
    std::vector<Field> fields;
    std::string ttlCol;          // SchemaProp.ttl_col
    int64_t ttlDuration = 0;     // SchemaProp.ttl_duration
    int64_t getFieldIndex(const std::string& name) const {
        for (size_t i = 0; i < fields.size(); i++) {
            if (fields[i].name == name) return static_cast<int64_t>(i);
        }
        return -1;
    }
    SupportedType getFieldType(int64_t i) const {
        if (i < 0 || i >= static_cast<int64_t>(fields.size())) return UNKNOWN;
        return fields[i].type;
    }
    SupportedType getFieldType(const std::string& name) const { return getFieldType(getFieldIndex(name)); }
    size_t getNumFields() const { return fields.size(); }
};
using SchemaPtr = std::shared_ptr<const Schema>;

// -------------------------------------------------------------------------------------
//  RowReader — restates src/dataman/RowReader.{h,cpp,inl}
// -------------------------------------------------------------------------------------
enum class ResultType {                       // src/dataman/DataCommon.h
    SUCCEEDED = 0, E_NAME_NOT_FOUND = -1, E_INDEX_OUT_OF_RANGE = -2, E_INCOMPATIBLE_TYPE = -3,
    E_VALUE_OUT_OF_RANGE = -4, E_DATA_INVALID = -5,
};

inline bool strToBool(const std::string& s) {     // DataCommon.h strToBool
    return s == "Y" || s == "y" || s == "T" || s == "t" || s == "yes" || s == "Yes" ||
           s == "YES" || s == "true" || s == "True" || s == "TRUE";
}

// folly::decodeVarint semantics: LEB128, at most 10 bytes; a truncated varint is an error.
inline int32_t decodeVarint(const uint8_t* p, size_t avail, uint64_t& out) {
    uint64_t v = 0;
    size_t i = 0;
    int shift = 0;
    while (true) {
        if (i >= avail || i >= 10) return -1;
        uint8_t b = p[i++];
        v |= static_cast<uint64_t>(b & 0x7f) << shift;
        if (!(b & 0x80)) break;
        shift += 7;
    }
    out = v;
    return static_cast<int32_t>(i);
}
inline void encodeVarint(uint64_t v, std::string& out) {   // folly::encodeVarint
    while (v >= 0x80) { out.push_back(static_cast<char>((v & 0x7f) | 0x80)); v >>= 7; }
    out.push_back(static_cast<char>(v));
}

struct ErrOrVariant {
    ResultType err = ResultType::SUCCEEDED;
    Variant v;
    bool ok() const { return err == ResultType::SUCCEEDED; }
};

class RowReader {
 public:
    // RowReader::getSchemaVer (RowReader.cpp:171-196): -1 for empty / too short rows.
    static int32_t getSchemaVer(const std::string& row) {
        if (row.empty()) return -1;
        const uint8_t* it = reinterpret_cast<const uint8_t*>(row.data());
        size_t verBytes = *(it++) >> 5;
        int32_t ver = 0;
        if (verBytes > 0) {
            if (verBytes + 1 > row.size()) return -1;
            for (size_t i = 0; i < verBytes; i++) ver |= (uint32_t(*(it++)) << (8 * i));
        }
        return ver;
    }
    // Returns nullptr where the reference returns an empty RowReader (or LOG(FATAL)s on a bad
    // header in the constructor, RowReader.cpp:199-212 — treated here as "no reader").
    // the schema is borrowed: its owner (the schema registry, a response's schema map) outlives the reader;
    // any shared_ptr to a Schema is taken by reference (no reference-count traffic per row)
    template <class P, class = decltype(std::declval<const P&>().get())>
    static std::unique_ptr<RowReader> make(const std::string& row, const P& schema) {
        return make(row, static_cast<const Schema*>(schema.get()));
    }
    static std::unique_ptr<RowReader> make(const std::string& row, const Schema* schema) {
        if (!schema) return nullptr;
        std::unique_ptr<RowReader> r(new RowReader());
        r->schema_ = schema;
        r->row_ = &row;
        if (!r->processHeader(row)) return nullptr;
        return r;
    }
    // make() into an existing reader (its offset vectors keep their capacity): false where make() gives
    // null. The harness's graphd loop reads millions of rows; a reader per row was three allocations.
    static bool reset(RowReader& r, const std::string& row, const Schema* schema) {
        if (!schema) return false;
        r.schema_ = schema;
        r.row_ = &row;
        return r.processHeader(row);
    }
    RowReader() = default;

    const Schema* getSchema() const { return schema_; }
    int32_t numFields() const { return static_cast<int32_t>(schema_->getNumFields()); }

    ResultType getBool(int64_t index, bool& v) const {
        int64_t offset;
        auto rc = getOffset(index, offset);
        if (rc != ResultType::SUCCEEDED) return rc;
        switch (schema_->getFieldType(index)) {                     // RowReader.cpp:421-458
            case BOOL:
                if (offset >= static_cast<int64_t>(size_)) return ResultType::E_DATA_INVALID;
                v = data_[offset] != 0;
                return ResultType::SUCCEEDED;
            case INT: case TIMESTAMP: {
                int64_t iv; int32_t n = readInteger(offset, iv);
                if (n <= 0) return ResultType::E_DATA_INVALID;
                v = iv != 0; return ResultType::SUCCEEDED;
            }
            case STRING: {
                std::string s; int32_t n = readString(offset, s);
                if (n <= 0) return ResultType::E_DATA_INVALID;
                v = strToBool(s); return ResultType::SUCCEEDED;
            }
            default: return ResultType::E_INCOMPATIBLE_TYPE;
        }
    }
    ResultType getInt(int64_t index, int64_t& v) const {             // RowReader.inl:27-57
        int64_t offset;
        auto rc = getOffset(index, offset);
        if (rc != ResultType::SUCCEEDED) return rc;
        switch (schema_->getFieldType(index)) {
            case INT: case TIMESTAMP: {
                int32_t n = readInteger(offset, v);
                if (n < 0) return ResultType::E_DATA_INVALID;
                return ResultType::SUCCEEDED;
            }
            default: return ResultType::E_INCOMPATIBLE_TYPE;
        }
    }
    ResultType getFloat(int64_t index, float& v) const {             // RowReader.cpp:461-488
        int64_t offset;
        auto rc = getOffset(index, offset);
        if (rc != ResultType::SUCCEEDED) return rc;
        switch (schema_->getFieldType(index)) {
            case FLOAT:
                if (offset + 4 > static_cast<int64_t>(size_)) return ResultType::E_DATA_INVALID;
                std::memcpy(&v, data_ + offset, 4); return ResultType::SUCCEEDED;
            case DOUBLE: {
                if (offset + 8 > static_cast<int64_t>(size_)) return ResultType::E_DATA_INVALID;
                double d; std::memcpy(&d, data_ + offset, 8); v = static_cast<float>(d);
                return ResultType::SUCCEEDED;
            }
            default: return ResultType::E_INCOMPATIBLE_TYPE;
        }
    }
    ResultType getDouble(int64_t index, double& v) const {           // RowReader.cpp:491-518
        int64_t offset;
        auto rc = getOffset(index, offset);
        if (rc != ResultType::SUCCEEDED) return rc;
        switch (schema_->getFieldType(index)) {
            case FLOAT: {
                if (offset + 4 > static_cast<int64_t>(size_)) return ResultType::E_DATA_INVALID;
                float f; std::memcpy(&f, data_ + offset, 4); v = static_cast<double>(f);
                return ResultType::SUCCEEDED;
            }
            case DOUBLE:
                if (offset + 8 > static_cast<int64_t>(size_)) return ResultType::E_DATA_INVALID;
                std::memcpy(&v, data_ + offset, 8); return ResultType::SUCCEEDED;
            default: return ResultType::E_INCOMPATIBLE_TYPE;
        }
    }
    ResultType getString(int64_t index, std::string& v) const {      // RowReader.cpp:521-539
        int64_t offset;
        auto rc = getOffset(index, offset);
        if (rc != ResultType::SUCCEEDED) return rc;
        if (schema_->getFieldType(index) != STRING) return ResultType::E_INCOMPATIBLE_TYPE;
        int32_t n = readString(offset, v);
        if (n < 0) return ResultType::E_DATA_INVALID;
        return ResultType::SUCCEEDED;
    }
    ResultType getVid(int64_t index, int64_t& v) const {             // RowReader.cpp:542-578
        int64_t offset;
        auto rc = getOffset(index, offset);
        if (rc != ResultType::SUCCEEDED) return rc;
        switch (schema_->getFieldType(index)) {
            case INT: case TIMESTAMP: {
                if (schema_->getFieldType(index) == TIMESTAMP) return ResultType::E_INCOMPATIBLE_TYPE;
                int32_t n = readInteger(offset, v);
                if (n < 0) return ResultType::E_DATA_INVALID;
                return ResultType::SUCCEEDED;
            }
            case VID:
                if (offset + 8 > static_cast<int64_t>(size_)) return ResultType::E_DATA_INVALID;
                std::memcpy(&v, data_ + offset, 8); return ResultType::SUCCEEDED;
            default: return ResultType::E_INCOMPATIBLE_TYPE;
        }
    }

    // RowReader::getPropByName (RowReader.h:136-193)
    static ErrOrVariant getPropByName(const RowReader* r, const std::string& prop) {
        ErrOrVariant out;
        int64_t idx = r->schema_->getFieldIndex(prop);
        SupportedType t = r->schema_->getFieldType(idx);             // = getFieldType(prop): one name scan
        if (idx < 0 && t == UNKNOWN) {
            // unknown name: getFieldType => kInvalidValueType => default case => E_DATA_INVALID
            out.err = ResultType::E_DATA_INVALID;
            return out;
        }
        switch (t) {
            case BOOL: { bool v = false; out.err = r->getBool(idx, v); out.v = v; break; }
            case INT: case TIMESTAMP: { int64_t v = 0; out.err = r->getInt(idx, v); out.v = v; break; }
            case VID: { int64_t v = 0; out.err = r->getVid(idx, v); out.v = v; break; }
            case FLOAT: { float v = 0; out.err = r->getFloat(idx, v); out.v = static_cast<double>(v); break; }
            case DOUBLE: { double v = 0; out.err = r->getDouble(idx, v); out.v = v; break; }
            case STRING: { std::string v; out.err = r->getString(idx, v); out.v = std::move(v); break; }
            default: out.err = ResultType::E_DATA_INVALID; break;
        }
        return out;
    }
    // RowReader::getDefaultProp (RowReader.h:111-134)
    static StatusOr<Variant> getDefaultProp(SupportedType type) {
        switch (type) {
            case BOOL: return Variant(false);
            case TIMESTAMP: case INT: return Variant(int64_t(0));
            case VID: return Variant(int64_t(0));
            case FLOAT: case DOUBLE: return Variant(0.0);
            case STRING: return Variant(std::string(""));
            default: return Status::Error("Unknown type");
        }
    }
    static StatusOr<Variant> getDefaultProp(const Schema* schema, const std::string& prop) {
        return getDefaultProp(schema->getFieldType(prop));
    }

 private:
    const Schema* schema_ = nullptr;
    const std::string* row_ = nullptr;
    const uint8_t* data_ = nullptr;
    size_t size_ = 0;
    int32_t headerLen_ = 0;
    int32_t numBytesForOffset_ = 0;
    mutable std::vector<std::pair<int64_t, uint8_t>> blockOffsets_;
    mutable std::vector<int64_t> offsets_;

    bool processHeader(const std::string& row) {                    // RowReader.cpp:215-260
        if (row.empty()) return false;
        const uint8_t* base = reinterpret_cast<const uint8_t*>(row.data());
        const uint8_t* it = base;
        numBytesForOffset_ = (*it & 0x07) + 1;
        int32_t verBytes = *(it++) >> 5;
        it += verBytes;
        uint32_t numFields = static_cast<uint32_t>(schema_->getNumFields());
        uint32_t numOffsets = (numFields >> 4);
        if (static_cast<size_t>(numBytesForOffset_) * numOffsets + verBytes + 1 > row.size()) return false;
        offsets_.assign(numFields + 1, -1);
        offsets_[0] = 0;
        blockOffsets_.clear();
        blockOffsets_.emplace_back(0, 0);
        for (uint32_t i = 0; i < numOffsets; i++) {
            int64_t offset = 0;
            for (int32_t j = 0; j < numBytesForOffset_; j++) offset |= (uint64_t(*(it++)) << (8 * j));
            blockOffsets_.emplace_back(offset, 0);
            offsets_[16 * (i + 1)] = offset;
        }
        headerLen_ = static_cast<int32_t>(it - base);
        offsets_[numFields] = static_cast<int64_t>(row.size()) - headerLen_;
        data_ = base + headerLen_;
        size_ = row.size() - headerLen_;
        return true;
    }
    int32_t readInteger(int64_t offset, int64_t& v) const {          // RowReader.inl:60-69
        if (offset < 0 || offset > static_cast<int64_t>(size_)) return -1;
        uint64_t u;
        int32_t n = decodeVarint(data_ + offset, size_ - offset, u);
        if (n < 0) return -1;
        v = static_cast<int64_t>(u);
        return n;
    }
    int32_t readString(int64_t offset, std::string& v) const {       // RowReader.cpp:390-401
        int64_t len;
        int32_t n = readInteger(offset, len);
        if (n <= 0) return -1;
        if (offset + n + len > static_cast<int64_t>(size_) || len < 0) return -1;
        v.assign(reinterpret_cast<const char*>(data_ + offset + n), static_cast<size_t>(len));
        return n + static_cast<int32_t>(len);
    }
    int64_t skipToNext(int64_t index, int64_t offset) const {        // RowReader.cpp:273-338
        if (offsets_[index + 1] >= 0) return offsets_[index + 1];
        switch (schema_->getFieldType(index)) {
            case BOOL: offset++; break;
            case INT: case TIMESTAMP: {
                int64_t v; int32_t len = readInteger(offset, v);
                if (len <= 0) return static_cast<int64_t>(ResultType::E_DATA_INVALID);
                offset += len; break;
            }
            case FLOAT: offset += 4; break;
            case DOUBLE: offset += 8; break;
            case STRING: {
                int64_t strLen; int32_t intLen = readInteger(offset, strLen);
                if (intLen <= 0) return static_cast<int64_t>(ResultType::E_DATA_INVALID);
                offset += intLen + strLen; break;
            }
            case VID: offset += 8; break;
            default: return static_cast<int64_t>(ResultType::E_DATA_INVALID);
        }
        if (offset > static_cast<int64_t>(size_)) return static_cast<int64_t>(ResultType::E_DATA_INVALID);
        offsets_[index + 1] = offset;
        int32_t base = static_cast<int32_t>((index + 1) >> 4);
        blockOffsets_[base].second = static_cast<uint8_t>((index + 1) & 0x0F);
        return offset;
    }
    int64_t skipToField(int64_t index) const {                       // RowReader.cpp:341-365
        if (index >= static_cast<int64_t>(schema_->getNumFields())) {
            return static_cast<int64_t>(ResultType::E_INDEX_OUT_OF_RANGE);
        }
        int64_t base = index >> 4;
        const auto& blockOffset = blockOffsets_[base];
        base <<= 4;
        int64_t maxVisitedIndex = base + blockOffset.second;
        if (index <= maxVisitedIndex) return offsets_[index];
        int64_t offset = offsets_[maxVisitedIndex];
        for (int64_t i = maxVisitedIndex; i < base + (index & 0x0f); i++) {
            offset = skipToNext(i, offset);
            if (offset < 0) return static_cast<int64_t>(ResultType::E_DATA_INVALID);
        }
        return offset;
    }
    ResultType getOffset(int64_t index, int64_t& offset) const {    // RR_GET_OFFSET
        if (index < 0) return ResultType::E_INDEX_OUT_OF_RANGE;
        offset = skipToField(index);
        if (offset < 0) return static_cast<ResultType>(offset);
        if (index >= static_cast<int64_t>(schema_->getNumFields())) return ResultType::E_INDEX_OUT_OF_RANGE;
        return ResultType::SUCCEEDED;
    }
};

// -------------------------------------------------------------------------------------
//  RowWriter — restates src/dataman/RowWriter.{h,cpp,inl}. With a schema, values are converted
//  to the column type (unmatched types write a type default); without one, the schema grows
//  with each written value (version 0). Block offsets every 16 fields, including the Skip()
//  bookkeeping exactly as RowWriter.cpp:213-263 does it.
// -------------------------------------------------------------------------------------
class RowWriter {
 public:
    // the schema is borrowed (see RowReader::make); without one the writer owns the schema it grows
    explicit RowWriter(const Schema* schema = nullptr) : schema_(schema) {
        if (!schema_) { own_ = std::make_shared<Schema>(); schema_ = own_.get(); }
    }
    template <class P, class = decltype(std::declval<const P&>().get())>
    explicit RowWriter(const P& schema) : RowWriter(static_cast<const Schema*>(schema.get())) {}
    RowWriter(const RowWriter& o) : schema_(o.own_ ? nullptr : o.schema_), own_(o.own_ ? std::make_shared<Schema>(*o.own_) : nullptr),
                                    cord_(o.cord_), colNum_(o.colNum_), blockOffsets_(o.blockOffsets_) {
        if (own_) schema_ = own_.get();
    }
    RowWriter& operator=(const RowWriter&) = delete;
    const Schema& schema() const { return *schema_; }

    RowWriter& operator<<(bool v) {
        SupportedType t = colType(BOOL);
        if (t == BOOL) cord_.push_back(static_cast<char>(v ? 1 : 0));
        else cord_.push_back(0);
        cleanUp(BOOL);
        return *this;
    }
    RowWriter& operator<<(float v) {
        SupportedType t = colType(FLOAT);
        if (t == FLOAT) putRaw(v);
        else if (t == DOUBLE) putRaw(static_cast<double>(v));
        else putRaw(static_cast<float>(0.0));
        cleanUp(FLOAT);
        return *this;
    }
    RowWriter& operator<<(double v) {
        SupportedType t = colType(DOUBLE);
        if (t == FLOAT) putRaw(static_cast<float>(v));
        else if (t == DOUBLE) putRaw(v);
        else putRaw(static_cast<double>(0.0));
        cleanUp(DOUBLE);
        return *this;
    }
    RowWriter& operator<<(int64_t v) { return writeIntegral(static_cast<uint64_t>(v)); }
    RowWriter& operator<<(int32_t v) { return writeIntegral(static_cast<uint64_t>(static_cast<int64_t>(v))); }
    RowWriter& operator<<(uint64_t v) { return writeIntegral(v); }
    RowWriter& operator<<(const std::string& v) {
        SupportedType t = colType(STRING);
        if (t == STRING) { encodeVarint(v.size(), cord_); cord_.append(v); }
        else encodeVarint(0, cord_);
        cleanUp(STRING);
        return *this;
    }
    RowWriter& operator<<(const char* v) { return operator<<(std::string(v)); }

    // RowWriter::operator<<(Skip) (RowWriter.cpp:213-263), including its block-offset check on i.
    void skip(int64_t toSkip) {
        if (toSkip <= 0) return;
        int32_t skipTo = static_cast<int32_t>(std::min<int64_t>(colNum_ + toSkip, schema_->getNumFields()));
        for (int i = static_cast<int>(colNum_); i < skipTo; i++) {
            switch (schema_->getFieldType(i)) {
                case BOOL: cord_.push_back(0); break;
                case INT: case TIMESTAMP: encodeVarint(0, cord_); break;
                case FLOAT: putRaw(static_cast<float>(0.0)); break;
                case DOUBLE: putRaw(static_cast<double>(0.0)); break;
                case STRING: encodeVarint(0, cord_); break;
                case VID: putRaw(static_cast<uint64_t>(0)); break;
                default: break;
            }
            if (i != 0 && (i >> 4 << 4) == i) blockOffsets_.push_back(static_cast<int64_t>(cord_.size()));
        }
        colNum_ = skipTo;
    }

    std::string encode() {                                          // RowWriter.cpp:48-87
        if (!own_) skip(static_cast<int64_t>(schema_->getNumFields()) - colNum_);
        std::string out;
        int64_t offsetBytes = calcOccupiedBytes(cord_.size());
        char header = static_cast<char>(offsetBytes - 1);
        SchemaVer ver = schema_->ver;
        if (ver > 0) {
            int64_t verBytes = calcOccupiedBytes(static_cast<uint64_t>(ver));
            header = static_cast<char>(header | (verBytes << 5));
            out.push_back(header);
            out.append(reinterpret_cast<const char*>(&ver), static_cast<size_t>(verBytes));
        } else {
            out.push_back(header);
        }
        for (auto off : blockOffsets_) out.append(reinterpret_cast<const char*>(&off), static_cast<size_t>(offsetBytes));
        out.append(cord_);
        return out;
    }
    int64_t size() const {                                          // RowWriter.cpp:27-37
        int64_t offsetBytes = calcOccupiedBytes(cord_.size());
        int64_t verBytes = 0;
        if (schema_->ver > 0) verBytes = calcOccupiedBytes(static_cast<uint64_t>(schema_->ver));
        return static_cast<int64_t>(cord_.size()) + offsetBytes * static_cast<int64_t>(blockOffsets_.size()) + verBytes + 1;
    }

 private:
    const Schema* schema_;
    std::shared_ptr<Schema> own_;       // set when writing without a schema (SchemaWriter)
    std::string cord_;
    int64_t colNum_ = 0;
    std::vector<int64_t> blockOffsets_;

    template <typename T>
    void putRaw(T v) { cord_.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
    static int64_t calcOccupiedBytes(uint64_t v) {
        int64_t bytes = 0;
        do { bytes++; v >>= 8; } while (v);
        return bytes;
    }
    SupportedType colType(SupportedType streamType) {               // RW_GET_COLUMN_TYPE
        if (colNum_ >= static_cast<int64_t>(schema_->getNumFields())) return streamType;
        return schema_->getFieldType(colNum_);
    }
    void cleanUp(SupportedType streamType) {                        // RW_CLEAN_UP_WRITE
        colNum_++;
        if (colNum_ != 0 && (colNum_ >> 4 << 4) == colNum_) blockOffsets_.push_back(static_cast<int64_t>(cord_.size()));
        if (colNum_ > static_cast<int64_t>(schema_->getNumFields())) {
            own_->fields.push_back(Field{"Column" + std::to_string(colNum_), streamType});
        }
    }
    RowWriter& writeIntegral(uint64_t v) {                          // RowWriter.inl:9-34
        SupportedType t = colType(INT);
        if (t == INT || t == TIMESTAMP) encodeVarint(v, cord_);
        else if (t == VID) putRaw(v);
        else encodeVarint(0, cord_);
        cleanUp(INT);
        return *this;
    }
};

}  // namespace orc
