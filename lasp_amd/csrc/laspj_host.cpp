// Host side of the drop-in, native (what the NIF links; include/laspj.h "host dictionary").
//
// The device never sees terms: element and token slots are positions in a dictionary the
// host keeps, ordered by Erlang term order.  The NIF receives values as terms; the bulk
// path hands them over as their external term format (term_to_binary/1 images, which
// the device codec also reads and writes), so the dictionary works on ETF:
//   * a walker over ETF images (the subset on this path: integers incl. bignums, floats,
//     atoms in all four encodings, tuples, nil, STRING_EXT and LIST_EXT lists, binaries)
//     that finds each term's extent without decoding it;
//   * Erlang's term order over two images (number < atom < tuple < nil < list <
//     bitstring; numbers compared by value across integer / bignum / float; atoms by
//     name; tuples by arity then elements; lists element-wise with prefix smaller;
//     binaries byte-wise), replacing enif_compare;
//   * the dictionary: element images -> element slot, and per element slot token images
//     -> token slot (<= 64), append-only, hashed by image bytes; term-order permutations
//     are computed on export (laspj_dict_export: the arrays laspj_etf_dict_create takes);
//   * encode: OR-Set / G-Set payloads -> {p, r} cells / bit words over the dictionary,
//     rejecting a value that is not an orddict / ordset (keys must ascend strictly in
//     term order), and decode for the reverse direction of small calls.
// Pure host code: no GPU needed (the CPU test suite runs it).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "laspj_internal.h"

namespace {

// ------------------------------------------------------------------ ETF reading

enum : int {
    kSmallInt = 97, kInt = 98, kFloatOld = 99, kAtom = 100, kSmallTuple = 104,
    kLargeTuple = 105, kNil = 106, kString = 107, kList = 108, kBinary = 109,
    kSmallBig = 110, kLargeBig = 111, kNewFloat = 70, kSmallAtom = 115, kAtomUtf8 = 118,
    kSmallAtomUtf8 = 119
};

inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

// the extent of the term at p (no version byte); 0 if malformed / unsupported
size_t term_len(const uint8_t* p, size_t n, int depth = 0) {
    if (n < 1 || depth > 64) return 0;
    switch (p[0]) {
        case kSmallInt: return n >= 2 ? 2 : 0;
        case kInt: return n >= 5 ? 5 : 0;
        case kNewFloat: return n >= 9 ? 9 : 0;
        case kFloatOld: return n >= 32 ? 32 : 0;
        case kAtom:
        case kAtomUtf8: {
            if (n < 3) return 0;
            size_t l = 3 + be16(p + 1);
            return l <= n ? l : 0;
        }
        case kSmallAtom:
        case kSmallAtomUtf8: {
            if (n < 2) return 0;
            size_t l = 2 + p[1];
            return l <= n ? l : 0;
        }
        case kSmallBig: {
            if (n < 3) return 0;
            size_t l = 3 + p[1];
            return l <= n ? l : 0;
        }
        case kLargeBig: {
            if (n < 6) return 0;
            size_t l = 6 + (size_t)be32(p + 1);
            return l <= n ? l : 0;
        }
        case kNil: return 1;
        case kString: {
            if (n < 3) return 0;
            size_t l = 3 + be16(p + 1);
            return l <= n ? l : 0;
        }
        case kBinary: {
            if (n < 5) return 0;
            size_t l = 5 + (size_t)be32(p + 1);
            return l <= n ? l : 0;
        }
        case kSmallTuple:
        case kLargeTuple: {
            const bool small = p[0] == kSmallTuple;
            if (n < (small ? 2u : 5u)) return 0;
            uint64_t ar = small ? p[1] : be32(p + 1);
            size_t off = small ? 2 : 5;
            for (uint64_t i = 0; i < ar; ++i) {
                size_t l = term_len(p + off, n - off, depth + 1);
                if (!l) return 0;
                off += l;
            }
            return off;
        }
        case kList: {
            if (n < 5) return 0;
            uint64_t cnt = be32(p + 1);
            size_t off = 5;
            for (uint64_t i = 0; i <= cnt; ++i) {      // elements, then the tail
                size_t l = term_len(p + off, n - off, depth + 1);
                if (!l) return 0;
                off += l;
            }
            return off;
        }
        default: return 0;
    }
}

int term_class(uint8_t tag) {
    switch (tag) {
        case kSmallInt: case kInt: case kSmallBig: case kLargeBig: case kNewFloat: case kFloatOld:
            return 0;
        case kAtom: case kSmallAtom: case kAtomUtf8: case kSmallAtomUtf8: return 1;
        case kSmallTuple: case kLargeTuple: return 6;
        case kNil: return 8;
        case kString: case kList: return 9;
        case kBinary: return 10;
        default: return -1;
    }
}

// a number: an exact integer (sign + little-endian magnitude) or a double
struct Num {
    bool is_float = false;
    double f = 0;
    int sign = 0;                 // -1, 0, 1
    std::vector<uint8_t> mag;     // little-endian, no high zero bytes
};

Num read_num(const uint8_t* p) {
    Num x;
    auto set_int = [&](int64_t v) {
        x.sign = v < 0 ? -1 : (v > 0 ? 1 : 0);
        uint64_t m = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
        while (m) {
            x.mag.push_back((uint8_t)m);
            m >>= 8;
        }
    };
    switch (p[0]) {
        case kSmallInt: set_int(p[1]); break;
        case kInt: set_int((int32_t)be32(p + 1)); break;
        case kSmallBig:
        case kLargeBig: {
            const bool small = p[0] == kSmallBig;
            size_t len = small ? p[1] : be32(p + 1);
            const uint8_t* s = p + (small ? 2 : 5);
            x.mag.assign(s + 1, s + 1 + len);
            while (!x.mag.empty() && x.mag.back() == 0) x.mag.pop_back();
            x.sign = x.mag.empty() ? 0 : (s[0] ? -1 : 1);
            break;
        }
        case kNewFloat: {
            uint64_t b = 0;
            for (int i = 0; i < 8; ++i) b = (b << 8) | p[1 + i];
            memcpy(&x.f, &b, 8);
            x.is_float = true;
            break;
        }
        case kFloatOld: {
            char buf[32];
            memcpy(buf, p + 1, 31);
            buf[31] = 0;
            x.f = strtod(buf, nullptr);
            x.is_float = true;
            break;
        }
    }
    return x;
}

int cmp_mag(const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {
    if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
    for (size_t i = a.size(); i-- > 0;)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return 0;
}

// integer vs double, exactly: through long double while the integer fits 64 bits (a
// long double holds a uint64 exactly, and every double converts exactly); beyond that
// by bit length, then the double's integral magnitude against the bignum's
int cmp_int_float(const Num& i, double f) {
    if (std::isnan(f)) return -1;
    if (std::isinf(f)) return f > 0 ? -1 : 1;
    long double fi;
    if (i.mag.size() <= 8) {
        uint64_t m = 0;
        for (size_t k = i.mag.size(); k-- > 0;) m = (m << 8) | i.mag[k];
        fi = (long double)m;
    } else {
        const int fs = f < 0 ? -1 : (f > 0 ? 1 : 0);
        if (i.sign != fs) return i.sign < fs ? -1 : 1;
        int bits = 8 * (int)(i.mag.size() - 1);
        for (uint8_t top = i.mag.back(); top; top >>= 1) ++bits;
        int ex = 0;
        const double m = std::frexp(std::fabs(f), &ex);   // |f| = m 2^ex, m in [0.5, 1)
        if (bits != ex) return ((bits < ex) == (i.sign > 0)) ? -1 : 1;
        // same bit length (> 64, so |f| >= 2^64 is an integer): |f| = mant << (ex - 53)
        const uint64_t mant = (uint64_t)std::ldexp(m, 53);
        const int sh = ex - 53;
        std::vector<uint8_t> fm(i.mag.size() + 1, 0);
        for (int k = 0; k < 8; ++k) {
            const unsigned v = (unsigned)((mant >> (8 * k)) & 0xFF) << (sh % 8);
            const size_t at = (size_t)(k + sh / 8);
            if (at < fm.size()) fm[at] |= (uint8_t)v;
            if (at + 1 < fm.size()) fm[at + 1] |= (uint8_t)(v >> 8);
        }
        while (!fm.empty() && fm.back() == 0) fm.pop_back();
        const int c = cmp_mag(i.mag, fm);
        return i.sign > 0 ? c : -c;
    }
    if (i.sign < 0) fi = -fi;
    const long double lf = f;
    return fi < lf ? -1 : (fi > lf ? 1 : 0);
}

int cmp_num(const uint8_t* a, const uint8_t* b) {
    // integers that fit 32 bits (SMALL_INTEGER_EXT / INTEGER_EXT): no decoding needed
    if ((a[0] == kSmallInt || a[0] == kInt) && (b[0] == kSmallInt || b[0] == kInt)) {
        const int64_t x = a[0] == kSmallInt ? a[1] : (int32_t)be32(a + 1);
        const int64_t y = b[0] == kSmallInt ? b[1] : (int32_t)be32(b + 1);
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    Num x = read_num(a), y = read_num(b);
    if (x.is_float && y.is_float) return x.f < y.f ? -1 : (x.f > y.f ? 1 : 0);
    if (!x.is_float && !y.is_float) {
        if (x.sign != y.sign) return x.sign < y.sign ? -1 : 1;
        int c = cmp_mag(x.mag, y.mag);
        return x.sign >= 0 ? c : -c;
    }
    if (!x.is_float) return cmp_int_float(x, y.f);
    return -cmp_int_float(y, x.f);
}

// an atom's name as UTF-8 (ATOM_EXT / SMALL_ATOM_EXT are latin-1)
std::string atom_name(const uint8_t* p) {
    const bool small = p[0] == kSmallAtom || p[0] == kSmallAtomUtf8;
    const bool utf8 = p[0] == kAtomUtf8 || p[0] == kSmallAtomUtf8;
    size_t len = small ? p[1] : be16(p + 1);
    const uint8_t* s = p + (small ? 2 : 3);
    if (utf8) return std::string((const char*)s, len);
    std::string out;
    for (size_t i = 0; i < len; ++i) {
        if (s[i] < 0x80) out.push_back((char)s[i]);
        else {
            out.push_back((char)(0xC0 | (s[i] >> 6)));
            out.push_back((char)(0x80 | (s[i] & 0x3F)));
        }
    }
    return out;
}

// 1 for the atom `true`, 0 for `false` (any of the four atom encodings), else -1
int bool_atom(const uint8_t* p) {
    const uint8_t* s;
    size_t len;
    if (p[0] == kAtom || p[0] == kAtomUtf8) {
        len = be16(p + 1);
        s = p + 3;
    } else if (p[0] == kSmallAtom || p[0] == kSmallAtomUtf8) {
        len = p[1];
        s = p + 2;
    } else {
        return -1;
    }
    if (len == 4 && !memcmp(s, "true", 4)) return 1;
    if (len == 5 && !memcmp(s, "false", 5)) return 0;
    return -1;
}

// elements of a list image, STRING_EXT or LIST_EXT (each STRING_EXT byte stands for a
// SMALL_INTEGER_EXT element)
struct ListIt {
    const uint8_t* p;
    size_t n;
    bool str;
    uint64_t count, i = 0;
    size_t off;
    uint8_t tmp[2];
    explicit ListIt(const uint8_t* img, size_t len) : p(img), n(len) {
        str = img[0] == kString;
        count = str ? be16(img + 1) : be32(img + 1);
        off = str ? 3 : 5;
    }
    // the next element's image, or nullptr at the end
    const uint8_t* next(size_t* len) {
        if (i >= count) return nullptr;
        ++i;
        if (str) {
            tmp[0] = kSmallInt;
            tmp[1] = p[off++];
            *len = 2;
            return tmp;
        }
        const uint8_t* e = p + off;
        *len = term_len(e, n - off);
        off += *len;
        return e;
    }
    const uint8_t* tail() const { return str ? nullptr : p + off; }
};

int term_cmp(const uint8_t* a, size_t na, const uint8_t* b, size_t nb, bool* ok) {
    const int ca = term_class(a[0]), cb = term_class(b[0]);
    if (ca < 0 || cb < 0) {
        *ok = false;
        return 0;
    }
    if (ca != cb) return ca < cb ? -1 : 1;
    switch (ca) {
        case 0: return cmp_num(a, b);
        case 1: {
            std::string x = atom_name(a), y = atom_name(b);
            int c = x.compare(y);
            return c < 0 ? -1 : (c > 0 ? 1 : 0);
        }
        case 6: {
            const bool sa = a[0] == kSmallTuple, sb = b[0] == kSmallTuple;
            uint64_t ra = sa ? a[1] : be32(a + 1), rb = sb ? b[1] : be32(b + 1);
            if (ra != rb) return ra < rb ? -1 : 1;
            size_t oa = sa ? 2 : 5, ob = sb ? 2 : 5;
            for (uint64_t k = 0; k < ra; ++k) {
                size_t la = term_len(a + oa, na - oa), lb = term_len(b + ob, nb - ob);
                int c = term_cmp(a + oa, la, b + ob, lb, ok);
                if (c || !*ok) return c;
                oa += la;
                ob += lb;
            }
            return 0;
        }
        case 8: return 0;
        case 9: {
            ListIt x(a, na), y(b, nb);
            for (;;) {
                size_t la = 0, lb = 0;
                const uint8_t* ea = x.next(&la);
                const uint8_t* eb = y.next(&lb);
                if (!ea || !eb) {
                    // proper lists only: a non-nil tail is outside this path
                    const uint8_t* ta = x.tail();
                    const uint8_t* tb = y.tail();
                    if ((!ea && ta && ta[0] != kNil) || (!eb && tb && tb[0] != kNil)) *ok = false;
                    if (!ea && !eb) return 0;
                    return !ea ? -1 : 1;     // a proper prefix is smaller
                }
                int c = term_cmp(ea, la, eb, lb, ok);
                if (c || !*ok) return c;
            }
        }
        case 10: {
            uint32_t la = be32(a + 1), lb = be32(b + 1);
            int c = memcmp(a + 5, b + 5, std::min(la, lb));
            if (c) return c < 0 ? -1 : 1;
            return la < lb ? -1 : (la > lb ? 1 : 0);
        }
    }
    *ok = false;
    return 0;
}

// ------------------------------------------------------------------ `==` classes

// A serialisation of the term at p in which two terms are byte-equal iff they compare
// equal (term_cmp == 0, Erlang's `==`): numbers by value (an integral float as the
// integer it equals, exactly as cmp_int_float compares them; -0.0 as 0), integers
// without regard to their encoding (SMALL_INTEGER / INTEGER / SMALL_BIG / LARGE_BIG),
// atoms by name whatever the encoding, STRING_EXT and LIST_EXT alike, [] however it is
// written.  The dictionary keys slots by image bytes, so `1` and `1.0` (or {a, 1} and
// {a, 1.0}) would take two slots where orddict:merge / ordsets:union see one key
// (SURVEY.md Appendix A): it hashes this form to find such pairs and refuses the second
// (LASPJ_DEC_EQUAL_TERMS).  False: a term outside this path.
bool canon(const uint8_t* p, size_t n, std::string* out, int depth = 0) {
    if (!n || depth > 64) return false;
    auto put32 = [&](uint64_t v) {
        for (int k = 3; k >= 0; --k) out->push_back((char)((v >> (8 * k)) & 0xFF));
    };
    auto put_int = [&](int sign, const uint8_t* mag, size_t len) {   // mag little-endian
        while (len && mag[len - 1] == 0) --len;
        out->push_back('I');
        out->push_back(len == 0 ? 0 : (sign < 0 ? '-' : '+'));
        put32(len);
        out->append((const char*)mag, len);
    };
    switch (term_class(p[0])) {
        case 0: {
            if (p[0] == kSmallInt || p[0] == kInt) {
                const int64_t v = p[0] == kSmallInt ? p[1] : (int32_t)be32(p + 1);
                uint64_t m = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
                uint8_t mag[8];
                for (int k = 0; k < 8; ++k) mag[k] = (uint8_t)(m >> (8 * k));
                put_int(v < 0 ? -1 : 1, mag, 8);
                return true;
            }
            Num x = read_num(p);
            if (!x.is_float) {
                put_int(x.sign, x.mag.data(), x.mag.size());
                return true;
            }
            const double f = x.f;
            if (!std::isfinite(f)) return false;
            if (f != std::trunc(f)) {
                uint64_t b;
                memcpy(&b, &f, 8);
                out->push_back('F');
                for (int k = 7; k >= 0; --k) out->push_back((char)((b >> (8 * k)) & 0xFF));
                return true;
            }
            // an integral double: |f| = mant 2^(ex-53), the integer's magnitude bytes
            int ex = 0;
            const double m = std::frexp(std::fabs(f), &ex);
            std::vector<uint8_t> mag((size_t)std::max(ex, 0) / 8 + 9, 0);
            if (ex > 0) {
                const uint64_t mant = (uint64_t)std::ldexp(m, 53);
                const int sh = ex - 53;
                if (sh >= 0) {
                    for (int k = 0; k < 8; ++k) {
                        const unsigned v = (unsigned)((mant >> (8 * k)) & 0xFF) << (sh % 8);
                        const size_t at = (size_t)(k + sh / 8);
                        if (at < mag.size()) mag[at] |= (uint8_t)v;
                        if (at + 1 < mag.size()) mag[at + 1] |= (uint8_t)(v >> 8);
                    }
                } else {
                    const uint64_t iv = mant >> (-sh);
                    for (int k = 0; k < 8; ++k) mag[k] = (uint8_t)(iv >> (8 * k));
                }
            }
            put_int(f < 0 ? -1 : 1, mag.data(), mag.size());
            return true;
        }
        case 1: {
            const std::string a = atom_name(p);
            out->push_back('A');
            put32(a.size());
            out->append(a);
            return true;
        }
        case 6: {
            const bool small = p[0] == kSmallTuple;
            const uint64_t ar = small ? p[1] : be32(p + 1);
            size_t off = small ? 2 : 5;
            out->push_back('T');
            put32(ar);
            for (uint64_t k = 0; k < ar; ++k) {
                const size_t l = term_len(p + off, n - off);
                if (!l || !canon(p + off, l, out, depth + 1)) return false;
                off += l;
            }
            return true;
        }
        case 8: out->push_back('N'); return true;
        case 9: {
            // [] written as an empty STRING_EXT / LIST_EXT is still []
            ListIt it(p, n);
            if (it.count == 0 && (it.str || (it.tail() && it.tail()[0] == kNil))) {
                out->push_back('N');
                return true;
            }
            out->push_back('L');
            put32(it.count);
            size_t el;
            while (const uint8_t* e = it.next(&el))
                if (!el || !canon(e, el, out, depth + 1)) return false;
            const uint8_t* t = it.tail();
            if (!t) {
                out->push_back('N');
                return true;
            }
            const size_t tl = term_len(t, n - (size_t)(t - p));
            return tl && canon(t, tl, out, depth + 1);
        }
        case 10: {
            const uint32_t l = be32(p + 1);
            out->push_back('B');
            put32(l);
            out->append((const char*)p + 5, l);
            return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------ dictionary

// images are stored once (a deque keeps their addresses); lookups hash the payload's
// own bytes in an open-addressing table (linear probing, 64-bit hashes kept beside the
// slots), so encoding allocates nothing and touches ~one cache line per lookup
inline uint64_t hash_bytes(const uint8_t* p, size_t n, uint64_t seed) {
    uint64_t h = seed ^ (n * 0x9E3779B97F4A7C15ull);
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        h = (h ^ v) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
        p += 8;
        n -= 8;
    }
    uint64_t v = 0;
    memcpy(&v, p, n);
    h = (h ^ v) * 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 29);
}

struct Table {
    struct Ent {
        uint64_t h;
        uint32_t owner;          // element slot for token keys, 0 for element keys
        uint32_t val;
        std::string_view key;
    };
    std::vector<Ent> ents;
    std::vector<uint32_t> idx;   // entry index + 1, 0 = empty
    uint64_t mask = 0;

    const Ent* find(uint64_t h, uint32_t owner, std::string_view key) const {
        if (idx.empty()) return nullptr;
        for (uint64_t i = h & mask;; i = (i + 1) & mask) {
            const uint32_t k = idx[i];
            if (!k) return nullptr;
            const Ent& e = ents[k - 1];
            if (e.h == h && e.owner == owner && e.key == key) return &e;
        }
    }
    // the first entry with this hash and owner for which same(key) holds
    template <class Same>
    const Ent* find_if(uint64_t h, uint32_t owner, Same same) const {
        if (idx.empty()) return nullptr;
        for (uint64_t i = h & mask;; i = (i + 1) & mask) {
            const uint32_t k = idx[i];
            if (!k) return nullptr;
            const Ent& e = ents[k - 1];
            if (e.h == h && e.owner == owner && same(e.key)) return &e;
        }
    }
    void grow() {
        const uint64_t cap = idx.empty() ? 1024 : idx.size() * 2;
        idx.assign(cap, 0);
        mask = cap - 1;
        for (uint32_t k = 0; k < ents.size(); ++k) {
            uint64_t i = ents[k].h & mask;
            while (idx[i]) i = (i + 1) & mask;
            idx[i] = k + 1;
        }
    }
    void insert(uint64_t h, uint32_t owner, std::string_view key, uint32_t val) {
        if (2 * (ents.size() + 1) > idx.size()) grow();
        ents.push_back(Ent{h, owner, val, key});
        uint64_t i = h & mask;
        while (idx[i]) i = (i + 1) & mask;
        idx[i] = (uint32_t)ents.size();
    }
    // undo the most recent insert.  Exact under linear probing when undone in LIFO order:
    // every later entry is gone already, and no earlier one probed past this slot.
    void pop_last() {
        const uint32_t k = (uint32_t)ents.size();
        uint64_t i = ents.back().h & mask;
        while (idx[i] != k) i = (i + 1) & mask;
        idx[i] = 0;
        ents.pop_back();
    }
};

constexpr uint64_t kElemSeed = 0x4C415350ull;

inline uint64_t tok_hash(uint32_t slot, const uint8_t* p, size_t n) {
    return hash_bytes(p, n, 0x9E3779B97F4A7C15ull * (slot + 1));
}

struct Dict {
    std::deque<std::string> store;
    std::vector<std::string_view> elems;
    std::vector<std::vector<std::string_view>> toks;
    Table elem_slot, tok_slot;
    // the `==` classes of the registered images (hash of canon(), owner as in the slot
    // tables; the key is the registered image, re-compared with term_cmp on a hash hit):
    // one image per class, so a slot never stands for half of an orddict key
    Table elem_eq, tok_eq;
    std::string scratch;
    // registrations of the payload being added (-1: an element, else the element slot of
    // a token), undone in reverse when the payload fails: binary_to_term/1 would have
    // rejected it whole, so none of its terms may take a slot
    std::vector<int64_t> journal;
    // token slots an element may hold: 64 (the columnar cells' {p, r} pair); a wide
    // namespace's dictionary (the NIF's k-pair cells) raises it
    uint32_t tok_cap = 64;
    // a wide dictionary's token images all have one length (its device templates are
    // fixed-width); 0: not wide, or no token yet
    uint32_t tok_len = 0, tok_len_max = 0;
    uint64_t ntok = 0;                      // tokens registered (all elements)
    uint32_t max_toks = 0;                  // most tokens of one element (an upper bound)
    // element slots that gained a token since the last dict_take_dirty (the NIF patches
    // their device rows; may repeat a slot or name one whose gain was rolled back)
    std::vector<uint32_t> dirty;
    // laspj_dict_export's term orders, kept between exports (registrations only append):
    // element slots sorted by term (the first ord_n slots), each element's token slots
    // sorted by term (valid while its size matches the element's token count)
    mutable std::vector<uint32_t> ord;
    mutable uint32_t ord_n = 0;
    mutable std::vector<std::vector<uint8_t>> tord;

    void rollback() {
        ord.clear();
        ord_n = 0;
        tord.clear();
        for (size_t j = journal.size(); j-- > 0;) {
            if (journal[j] < 0) {
                elem_slot.pop_last();
                elem_eq.pop_last();
                elems.pop_back();
                toks.pop_back();
            } else {
                tok_slot.pop_last();
                tok_eq.pop_last();
                toks[(size_t)journal[j]].pop_back();
                --ntok;
            }
            store.pop_back();
        }
        journal.clear();
        if (!ntok) tok_len = 0;             // (a length no registered token fixes)
    }

    std::string_view keep(const uint8_t* p, size_t n) {
        store.emplace_back((const char*)p, n);
        return std::string_view(store.back());
    }
    // element slot of an image, or -1
    int64_t elem(const uint8_t* k, size_t kl) const {
        const Table::Ent* e = elem_slot.find(hash_bytes(k, kl, kElemSeed), 0,
                                             std::string_view((const char*)k, kl));
        return e ? (int64_t)e->val : -1;
    }
    int tok(uint32_t es, const uint8_t* t, size_t tl) const {
        const Table::Ent* e = tok_slot.find(tok_hash(es, t, tl), es,
                                            std::string_view((const char*)t, tl));
        return e ? (int)e->val : -1;
    }
};

// the payload's term: after an optional <<Tag, Vers>> prefix and the version byte 131
int payload_term(const uint8_t* p, size_t n, int tag, int vers, const uint8_t** t, size_t* tn) {
    if (tag >= 0) {
        if (n < 2 || p[0] != (uint8_t)tag) return LASPJ_DEC_INVALID_BINARY;
        if (vers >= 0 && p[1] != (uint8_t)vers) return LASPJ_DEC_UNSUPPORTED_VERSION;
        p += 2;
        n -= 2;
    }
    if (n < 2 || p[0] != 131) return LASPJ_DEC_MALFORMED;
    size_t l = term_len(p + 1, n - 1);
    if (!l || l != n - 1) return LASPJ_DEC_MALFORMED;
    *t = p + 1;
    *tn = l;
    return LASPJ_DEC_OK;
}

// walk [{Elem, [{Tok, Bool}]}] in one pass (each byte read once, extents found as it
// goes): on_elem(elem image) per element, on_tok(elem image, tok image, flag) per token;
// *used = the term's length.  Returns a LASPJ_DEC_* status: the first problem in stream
// order (callers that need "not a term at all" to win re-check with term_len).
template <class OnElem, class OnTok>
int walk_orset(const uint8_t* t, size_t tn, size_t* used, OnElem on_elem, OnTok on_tok) {
    if (tn < 1) return LASPJ_DEC_MALFORMED;
    if (t[0] == kNil) {
        *used = 1;
        return LASPJ_DEC_OK;
    }
    if (t[0] != kList || tn < 5) return LASPJ_DEC_MALFORMED;
    const uint32_t cnt = be32(t + 1);
    size_t off = 5;
    for (uint32_t i = 0; i < cnt; ++i) {
        if (off + 2 > tn || t[off] != kSmallTuple || t[off + 1] != 2) return LASPJ_DEC_MALFORMED;
        off += 2;
        const uint8_t* k = t + off;
        const size_t kl = term_len(k, tn - off);
        if (!kl) return LASPJ_DEC_MALFORMED;
        off += kl;
        if (off >= tn) return LASPJ_DEC_MALFORMED;
        if (t[off] == kNil) return LASPJ_DEC_UNREPRESENTABLE;      // an element without tokens
        if (t[off] != kList || off + 5 > tn) return LASPJ_DEC_MALFORMED;
        const uint32_t m = be32(t + off + 1);
        off += 5;
        if (int st = on_elem(k, kl)) return st;
        for (uint32_t j = 0; j < m; ++j) {
            if (off + 2 > tn || t[off] != kSmallTuple || t[off + 1] != 2)
                return LASPJ_DEC_MALFORMED;
            off += 2;
            const uint8_t* tk = t + off;
            const size_t tkl = term_len(tk, tn - off);
            if (!tkl) return LASPJ_DEC_MALFORMED;
            off += tkl;
            const size_t fl = off < tn ? term_len(t + off, tn - off) : 0;
            if (!fl) return LASPJ_DEC_MALFORMED;
            const int flag = bool_atom(t + off);
            off += fl;
            if (flag < 0) return LASPJ_DEC_MALFORMED;
            if (int st = on_tok(k, kl, tk, tkl, flag == 1)) return st;
        }
        if (off >= tn || t[off] != kNil) return LASPJ_DEC_MALFORMED;   // proper token list
        off += 1;
    }
    if (off >= tn || t[off] != kNil) return LASPJ_DEC_MALFORMED;       // proper outer list
    *used = off + 1;
    return LASPJ_DEC_OK;
}

// the payload's term for the one-pass walker: after an optional <<Tag, Vers>> prefix and
// the version byte 131 (its extent is checked by the walk)
int payload_start(const uint8_t* p, size_t n, int tag, const uint8_t** t, size_t* tn) {
    if (tag >= 0) {
        if (n < 2 || p[0] != (uint8_t)tag) return LASPJ_DEC_INVALID_BINARY;
        p += 2;
        n -= 2;
    }
    if (n < 2 || p[0] != 131) return LASPJ_DEC_MALFORMED;
    *t = p + 1;
    *tn = n - 1;
    return LASPJ_DEC_OK;
}

// an OR-Set payload walked once; a term that is not well-formed ETF reports MALFORMED
// even when an earlier element already failed for another reason (binary_to_term/1
// rejects the whole payload first)
template <class OnElem, class OnTok>
int walk_orset_payload(const uint8_t* p, size_t n, int tag, OnElem on_elem, OnTok on_tok) {
    const uint8_t* t;
    size_t tn, used = 0;
    int st = payload_start(p, n, tag, &t, &tn);
    if (st) return st;
    st = walk_orset(t, tn, &used, on_elem, on_tok);
    if (st == LASPJ_DEC_OK) return used == tn ? LASPJ_DEC_OK : LASPJ_DEC_MALFORMED;
    if (st != LASPJ_DEC_MALFORMED && term_len(t, tn) != tn) return LASPJ_DEC_MALFORMED;
    return st;
}

template <class OnElem>
int walk_gset(const uint8_t* t, size_t tn, OnElem on_elem) {
    if (t[0] == kNil) return LASPJ_DEC_OK;
    if (t[0] != kList && t[0] != kString) return LASPJ_DEC_MALFORMED;
    ListIt it(t, tn);
    size_t el;
    while (const uint8_t* e = it.next(&el)) {
        // STRING_EXT elements are synthesised SMALL_INTEGER_EXT images (2 bytes)
        if (int st = on_elem(e, el)) return st;
    }
    if (it.tail() && it.tail()[0] != kNil) return LASPJ_DEC_MALFORMED;
    return LASPJ_DEC_OK;
}

// the `==` class hash of an image (canon), or false for a term outside this path
bool eq_hash(Dict* d, const uint8_t* k, size_t kl, uint64_t seed, uint64_t* h) {
    d->scratch.clear();
    if (!canon(k, kl, &d->scratch)) return false;
    *h = hash_bytes((const uint8_t*)d->scratch.data(), d->scratch.size(), seed);
    return true;
}

int reg_elem(Dict* d, const uint8_t* k, size_t kl, uint32_t* slot) {
    const int64_t f = d->elem(k, kl);
    if (f >= 0) {
        *slot = (uint32_t)f;
        return LASPJ_DEC_OK;
    }
    bool ok = true;
    term_cmp(k, kl, k, kl, &ok);              // the comparator must handle the term
    if (!ok) return LASPJ_DEC_MALFORMED;
    uint64_t he = 0;
    if (!eq_hash(d, k, kl, kElemSeed, &he)) return LASPJ_DEC_MALFORMED;
    // another image of an `==`-equal term already holds a slot (1 vs 1.0)
    if (d->elem_eq.find_if(he, 0, [&](std::string_view o) {
            bool ok2 = true;
            return term_cmp(k, kl, (const uint8_t*)o.data(), o.size(), &ok2) == 0 && ok2;
        }))
        return LASPJ_DEC_EQUAL_TERMS;
    if (d->elems.size() >= (1u << 24)) return LASPJ_DEC_UNREPRESENTABLE;
    *slot = (uint32_t)d->elems.size();
    std::string_view v = d->keep(k, kl);
    d->elem_slot.insert(hash_bytes(k, kl, kElemSeed), 0, v, *slot);
    d->elem_eq.insert(he, 0, v, *slot);
    d->elems.push_back(v);
    d->toks.emplace_back();
    d->journal.push_back(-1);
    return LASPJ_DEC_OK;
}

int reg_tok(Dict* d, uint32_t es, const uint8_t* t, size_t tl, uint16_t* slot) {
    const int f = d->tok(es, t, tl);
    if (f >= 0) {
        *slot = (uint16_t)f;
        return LASPJ_DEC_OK;
    }
    bool ok = true;
    term_cmp(t, tl, t, tl, &ok);
    if (!ok) return LASPJ_DEC_MALFORMED;
    uint64_t ht = 0;
    if (!eq_hash(d, t, tl, 0x9E3779B97F4A7C15ull * (es + 1), &ht)) return LASPJ_DEC_MALFORMED;
    if (d->tok_eq.find_if(ht, es, [&](std::string_view o) {
            bool ok2 = true;
            return term_cmp(t, tl, (const uint8_t*)o.data(), o.size(), &ok2) == 0 && ok2;
        }))
        return LASPJ_DEC_EQUAL_TERMS;
    if (d->toks[es].size() >= d->tok_cap) return LASPJ_DEC_UNREPRESENTABLE;
    if (d->tok_len_max) {
        if (d->tok_len ? tl != d->tok_len : tl > d->tok_len_max) return LASPJ_DEC_UNREPRESENTABLE;
        d->tok_len = (uint32_t)tl;
    }
    *slot = (uint16_t)d->toks[es].size();
    std::string_view v = d->keep(t, tl);
    d->tok_slot.insert(tok_hash(es, t, tl), es, v, *slot);
    d->tok_eq.insert(ht, es, v, *slot);
    d->toks[es].push_back(v);
    ++d->ntok;
    d->max_toks = std::max<uint32_t>(d->max_toks, (uint32_t)d->toks[es].size());
    d->journal.push_back((int64_t)es);
    d->dirty.push_back(es);
    return LASPJ_DEC_OK;
}

int cmp_view(std::string_view a, std::string_view b) {
    bool ok = true;
    return term_cmp((const uint8_t*)a.data(), a.size(), (const uint8_t*)b.data(), b.size(), &ok);
}

}  // namespace

struct laspj_dict {
    Dict d;
};

extern "C" {

int laspj_term_compare(const uint8_t* a, size_t na, const uint8_t* b, size_t nb, int* out) {
    if (!a || !b || !out || !na || !nb) return LASPJ_E_INVAL;
    // maps, pids, ports, references, funs, exports and bit strings: valid terms, but not
    // ones this path holds
    auto other = [](uint8_t t) {
        return t == 116 || t == 88 || t == 103 || t == 89 || t == 102 || t == 120 ||
               t == 90 || t == 114 || t == 101 || t == 112 || t == 117 || t == 113 || t == 77;
    };
    if (other(a[0]) || other(b[0])) return LASPJ_E_UNSUPPORTED;
    if (term_len(a, na) != na || term_len(b, nb) != nb) return LASPJ_E_INVAL;
    bool ok = true;
    int c = term_cmp(a, na, b, nb, &ok);
    if (!ok) return LASPJ_E_UNSUPPORTED;
    *out = c;
    return LASPJ_OK;
}

int laspj_dict_create(laspj_dict** out) {
    if (!out) return LASPJ_E_INVAL;
    *out = new (std::nothrow) laspj_dict;
    return *out ? LASPJ_OK : LASPJ_E_NOMEM;
}

int laspj_dict_destroy(laspj_dict* d) {
    if (!d) return LASPJ_E_INVAL;
    delete d;
    return LASPJ_OK;
}

int laspj_dict_add(laspj_dict* dict, int32_t kind, const uint8_t* blob, const uint64_t* offsets,
                   uint64_t n, int tag, int32_t* status) {
    if (!dict || (n && (!blob || !offsets || !status))) return LASPJ_E_INVAL;
    if (kind != LASPJ_KIND_ORSET && kind != LASPJ_KIND_GSET) return LASPJ_E_KIND;
    Dict* d = &dict->d;
    try {
        for (uint64_t i = 0; i < n; ++i) {
            if (offsets[i + 1] < offsets[i]) return LASPJ_E_INVAL;
            const uint8_t* pp = blob + offsets[i];
            const size_t pn = offsets[i + 1] - offsets[i];
            int st;
            d->journal.clear();
            if (kind == LASPJ_KIND_ORSET) {
                uint32_t cur = 0;
                st = walk_orset_payload(
                    pp, pn, tag, [&](const uint8_t* k, size_t kl) { return reg_elem(d, k, kl, &cur); },
                    [&](const uint8_t*, size_t, const uint8_t* tk, size_t tkl, bool) {
                        uint16_t s;
                        return reg_tok(d, cur, tk, tkl, &s);
                    });
            } else {
                const uint8_t* t;
                size_t tn;
                st = payload_term(pp, pn, tag, -1, &t, &tn);
                if (st == LASPJ_DEC_OK)
                    st = walk_gset(t, tn, [&](const uint8_t* e, size_t el) {
                        uint32_t s;
                        return reg_elem(d, e, el, &s);
                    });
            }
            if (st != LASPJ_DEC_OK) d->rollback();
            d->journal.clear();
            status[i] = st;
        }
    } catch (const std::bad_alloc&) {
        d->rollback();
        return LASPJ_E_NOMEM;
    }
    return LASPJ_OK;
}

int laspj_dict_info(const laspj_dict* dict, uint32_t* elements, uint64_t* elem_bytes,
                    uint64_t* tok_bytes) {
    if (!dict) return LASPJ_E_INVAL;
    const Dict& d = dict->d;
    uint64_t eb = 0, tb = 0;
    for (const auto& e : d.elems) eb += e.size();
    for (const auto& v : d.toks)
        for (const auto& t : v) tb += t.size();
    if (elements) *elements = (uint32_t)d.elems.size();
    if (elem_bytes) *elem_bytes = eb;
    if (tok_bytes) *tok_bytes = tb;
    return LASPJ_OK;
}

int laspj_dict_export(const laspj_dict* dict, uint32_t E, uint8_t* elem_blob, uint32_t* elem_off,
                      uint32_t* elem_order, uint8_t* tok_blob, uint32_t* tok_off,
                      uint8_t* tok_order) {
    if (!dict || !elem_off || !elem_order) return LASPJ_E_INVAL;
    const Dict& d = dict->d;
    const uint32_t K = (uint32_t)d.elems.size();
    if (E < K) return LASPJ_E_RANGE;
    try {
        // element images and offsets (E + 1), slots in term order, unused slots last
        uint64_t off = 0;
        elem_off[0] = 0;
        for (uint32_t e = 0; e < E; ++e) {
            if (e < K) {
                if (elem_blob) memcpy(elem_blob + off, d.elems[e].data(), d.elems[e].size());
                off += d.elems[e].size();
            }
            if (off > 0xFFFFFFFFull) return LASPJ_E_RANGE;
            elem_off[e + 1] = (uint32_t)off;
        }
        // the cached order of the first ord_n slots, the newer slots sorted and merged in
        // (ties keep slot order: std::merge takes the earlier range's element first)
        auto less = [&](uint32_t x, uint32_t y) { return cmp_view(d.elems[x], d.elems[y]) < 0; };
        if (d.ord_n > K) {
            d.ord.clear();
            d.ord_n = 0;
        }
        if (d.ord_n < K) {
            std::vector<uint32_t> add(K - d.ord_n);
            for (uint32_t e = d.ord_n; e < K; ++e) add[e - d.ord_n] = e;
            std::stable_sort(add.begin(), add.end(), less);
            std::vector<uint32_t> merged(K);
            std::merge(d.ord.begin(), d.ord.end(), add.begin(), add.end(), merged.begin(), less);
            d.ord.swap(merged);
            d.ord_n = K;
        }
        const std::vector<uint32_t>& ord = d.ord;
        for (uint32_t e = 0; e < E; ++e) elem_order[e] = e < K ? ord[e] : e;
        if (d.tord.size() > K) d.tord.clear();
        d.tord.resize(K);
        if (tok_off) {
            uint64_t to = 0;
            tok_off[0] = 0;
            for (uint32_t e = 0; e < E; ++e) {
                // the element's tokens, then its empty slots at the running offset
                uint32_t* te = tok_off + 64ull * e + 1;
                const uint32_t cnt = e < K ? (uint32_t)std::min<size_t>(d.toks[e].size(), 64) : 0u;
                for (uint32_t k = 0; k < cnt; ++k) {
                    const std::string_view t = d.toks[e][k];
                    if (tok_blob) memcpy(tok_blob + to, t.data(), t.size());
                    to += t.size();
                    if (to > 0xFFFFFFFFull) return LASPJ_E_RANGE;
                    te[k] = (uint32_t)to;
                }
                std::fill(te + cnt, te + 64, (uint32_t)to);
                if (tok_order) {
                    uint8_t* o = tok_order + 64ull * e;
                    memset(o, 0xFF, 64);
                    if (e < K) {
                        std::vector<uint8_t>& ts = d.tord[e];
                        if (ts.size() != d.toks[e].size()) {    // tokens added since
                            ts.resize(d.toks[e].size());
                            for (size_t k = 0; k < ts.size(); ++k) ts[k] = (uint8_t)k;
                            std::stable_sort(ts.begin(), ts.end(), [&](uint8_t x, uint8_t y) {
                                return cmp_view(d.toks[e][x], d.toks[e][y]) < 0;
                            });
                        }
                        memcpy(o, ts.data(), ts.size());
                    }
                }
            }
        }
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
    return LASPJ_OK;
}

int laspj_dict_encode(const laspj_dict* dict, int32_t kind, const uint8_t* blob,
                      const uint64_t* offsets, uint64_t n, int tag, uint32_t E, uint64_t* out,
                      int32_t* status) {
    return laspj::dict_encode_cells(dict, kind, blob, offsets, n, tag, E, 1, out, status);
}

}  // extern "C"

// (tw {p, r} pairs per OR-Set element: token slot f in pair f / 64 — a wide namespace)
int laspj::dict_encode_cells(const laspj_dict* dict, int32_t kind, const uint8_t* blob,
                             const uint64_t* offsets, uint64_t n, int tag, uint32_t E,
                             uint32_t tw, uint64_t* out, int32_t* status) {
    if (!dict || (n && (!blob || !offsets || !status || !out)) || tw == 0) return LASPJ_E_INVAL;
    if (kind != LASPJ_KIND_ORSET && kind != LASPJ_KIND_GSET) return LASPJ_E_KIND;
    const Dict& d = dict->d;
    const uint64_t wpr = kind == LASPJ_KIND_ORSET ? 2ull * E * tw : (E + 63ull) / 64ull;
    try {
        for (uint64_t i = 0; i < n; ++i) {
            if (offsets[i + 1] < offsets[i]) return LASPJ_E_INVAL;
            uint64_t* cells = out + i * wpr;
            memset(cells, 0, wpr * 8);
            const uint8_t* pp = blob + offsets[i];
            const size_t pn = offsets[i + 1] - offsets[i];
            int st;
            // keys must ascend strictly (an orddict / ordset), tokens likewise
            std::string_view prev_e, prev_t;
            bool have_e = false, have_t = false;
            uint32_t cur = 0;
            if (kind == LASPJ_KIND_ORSET) {
                st = walk_orset_payload(
                    pp, pn, tag,
                    [&](const uint8_t* k, size_t kl) -> int {
                        // k points into the payload: the view stays valid
                        std::string_view key((const char*)k, kl);
                        const int64_t f = d.elem(k, kl);
                        if (f < 0 || f >= (int64_t)E) return LASPJ_DEC_UNKNOWN_TERM;
                        if (have_e && cmp_view(prev_e, key) >= 0) return LASPJ_DEC_UNKNOWN_TERM;
                        prev_e = key;
                        have_e = true;
                        have_t = false;
                        cur = (uint32_t)f;
                        return LASPJ_DEC_OK;
                    },
                    [&](const uint8_t*, size_t, const uint8_t* tk, size_t tkl, bool flag) -> int {
                        std::string_view key((const char*)tk, tkl);
                        const int f = d.tok(cur, tk, tkl);
                        if (f < 0) return LASPJ_DEC_UNKNOWN_TERM;
                        if ((uint32_t)f >= 64u * tw) return LASPJ_DEC_UNREPRESENTABLE;
                        if (have_t && cmp_view(prev_t, key) >= 0) return LASPJ_DEC_UNKNOWN_TERM;
                        prev_t = key;
                        have_t = true;
                        uint64_t* pr = cells + 2ull * ((uint64_t)cur * tw + (uint32_t)f / 64u);
                        pr[0] |= 1ull << (f & 63);
                        if (flag) pr[1] |= 1ull << (f & 63);
                        return LASPJ_DEC_OK;
                    });
            } else {
                const uint8_t* t;
                size_t tn;
                std::string prev_buf;
                st = payload_term(pp, pn, tag, -1, &t, &tn);
                if (st == LASPJ_DEC_OK)
                    st = walk_gset(t, tn, [&](const uint8_t* k, size_t kl) -> int {
                        std::string_view key((const char*)k, kl);
                        const int64_t f = d.elem(k, kl);
                        if (f < 0 || f >= (int64_t)E) return LASPJ_DEC_UNKNOWN_TERM;
                        if (have_e && cmp_view(prev_e, key) >= 0) return LASPJ_DEC_UNKNOWN_TERM;
                        // a STRING_EXT element's image lives in the iterator's scratch: copy
                        // it (the buffer keeps its capacity, so this does not allocate)
                        prev_buf.assign(key.data(), key.size());
                        prev_e = prev_buf;
                        have_e = true;
                        cells[f >> 6] |= 1ull << (f & 63);
                        return LASPJ_DEC_OK;
                    });
            }
            if (st != LASPJ_DEC_OK) memset(cells, 0, wpr * 8);
            status[i] = st;
        }
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
    return LASPJ_OK;
}

// ------------------------------------------------------------------ internal accessors
// (laspj_internal.h): what laspj::etf_dict_patch reads from the host dictionary when the
// NIF path patches the device images of elements that gained tokens instead of
// rebuilding them
namespace laspj {

uint32_t dict_elements(const laspj_dict* dict) {
    return dict ? (uint32_t)dict->d.elems.size() : 0u;
}

void dict_take_dirty(laspj_dict* dict, std::vector<uint32_t>* out) {
    out->clear();
    if (dict) out->swap(dict->d.dirty);
}

uint32_t dict_max_tokens(const laspj_dict* dict) { return dict->d.max_toks; }

uint32_t dict_token_count(const laspj_dict* dict, uint32_t e) {
    if (!dict || e >= dict->d.toks.size()) return 0;
    return (uint32_t)dict->d.toks[e].size();
}

// element slot e's token images by slot, and its slots in term order (order[j] = the slot
// of the j-th smallest token): the same order laspj_dict_export writes (and caches)
bool dict_tokens(const laspj_dict* dict, uint32_t e, std::vector<std::string_view>* imgs,
                 std::vector<uint8_t>* order) {
    if (!dict || e >= dict->d.toks.size()) return false;
    const Dict& d = dict->d;
    const auto& tv = d.toks[e];
    imgs->assign(tv.begin(), tv.end());
    if (d.tord.size() < d.toks.size()) d.tord.resize(d.toks.size());
    std::vector<uint8_t>& ts = d.tord[e];
    if (ts.size() != tv.size()) {
        ts.resize(tv.size());
        for (size_t k = 0; k < ts.size(); ++k) ts[k] = (uint8_t)k;
        std::stable_sort(ts.begin(), ts.end(), [&](uint8_t x, uint8_t y) {
            return cmp_view(tv[x], tv[y]) < 0;
        });
    }
    *order = ts;
    return true;
}

// Register the terms of the OR-Set payload p[0, n) elements that start in [from, to)
// (from: an element's first byte, its 104 2 tuple header, as the segment decoder found
// it): the same per-element parse and registration as laspj_dict_add's walk, over a range
// — the NIF registers only the segments whose decode met an unknown term.  Stops at the
// outer list's closing nil.  On any failure the range's registrations are undone.
int dict_add_elems(laspj_dict* dict, const uint8_t* p, size_t n, size_t from, size_t to) {
    if (!dict || !p) return LASPJ_E_INVAL;
    Dict* d = &dict->d;
    d->journal.clear();
    int st = LASPJ_DEC_OK;
    try {
        size_t off = from;
        while (st == LASPJ_DEC_OK && off < to && off < n && p[off] != kNil) {
            if (off + 2 > n || p[off] != kSmallTuple || p[off + 1] != 2) {
                st = LASPJ_DEC_MALFORMED;
                break;
            }
            off += 2;
            const uint8_t* k = p + off;
            const size_t kl = term_len(k, n - off);
            if (!kl) { st = LASPJ_DEC_MALFORMED; break; }
            off += kl;
            if (off >= n) { st = LASPJ_DEC_MALFORMED; break; }
            if (p[off] == kNil) { st = LASPJ_DEC_UNREPRESENTABLE; break; }
            if (p[off] != kList || off + 5 > n) { st = LASPJ_DEC_MALFORMED; break; }
            const uint32_t m = be32(p + off + 1);
            off += 5;
            uint32_t cur = 0;
            if ((st = reg_elem(d, k, kl, &cur))) break;
            for (uint32_t j = 0; j < m && st == LASPJ_DEC_OK; ++j) {
                if (off + 2 > n || p[off] != kSmallTuple || p[off + 1] != 2) {
                    st = LASPJ_DEC_MALFORMED;
                    break;
                }
                off += 2;
                const uint8_t* tk = p + off;
                const size_t tkl = term_len(tk, n - off);
                if (!tkl) { st = LASPJ_DEC_MALFORMED; break; }
                off += tkl;
                const size_t fl = off < n ? term_len(p + off, n - off) : 0;
                if (!fl || bool_atom(p + off) < 0) { st = LASPJ_DEC_MALFORMED; break; }
                off += fl;
                uint16_t s;
                st = reg_tok(d, cur, tk, tkl, &s);
            }
            if (st) break;
            if (off >= n || p[off] != kNil) { st = LASPJ_DEC_MALFORMED; break; }
            off += 1;
        }
    } catch (const std::bad_alloc&) {
        d->rollback();
        d->journal.clear();
        return LASPJ_E_NOMEM;
    }
    if (st != LASPJ_DEC_OK) d->rollback();
    d->journal.clear();
    return st;
}

}  // namespace laspj

// ------------------------------------------------------------------ list values as images
// (laspj_list_etf.cpp): the combinator bodies and bind/3 on lists that are not orddicts /
// ordsets (lasp_core.erl:460-712) take and give term_to_binary images; these walk an image
// into list items over a host dictionary and write items back into an image.
namespace laspj {

namespace {

constexpr uint64_t kPairBit = 1ull << 62;
constexpr uint64_t kFlagBit = 1ull << 63;

void put_be32(std::string* o, uint32_t v) {
    for (int k = 3; k >= 0; --k) o->push_back((char)((v >> (8 * k)) & 0xFF));
}

bool small_int(std::string_view img, uint8_t* v) {
    if (img.size() == 2 && (uint8_t)img[0] == kSmallInt) {
        *v = (uint8_t)img[1];
        return true;
    }
    return false;
}

}  // namespace

int list_walk(laspj_dict* dict, int32_t kind, const uint8_t* p, size_t n, ListItems* it,
              std::vector<uint32_t>* args) {
    Dict* d = &dict->d;
    it->keys.clear();
    it->toff.assign(1, 0);
    it->toks.clear();
    d->journal.clear();
    int st = LASPJ_DEC_OK;
    try {
        const uint8_t* t;
        size_t tn;
        st = payload_term(p, n, -1, -1, &t, &tn);
        if (st == LASPJ_DEC_OK && t[0] != kNil && t[0] != kList && t[0] != kString)
            st = LASPJ_DEC_MALFORMED;                    // not a list
        if (st == LASPJ_DEC_OK && t[0] != kNil) {
            ListIt li(t, tn);
            size_t el;
            while (st == LASPJ_DEC_OK) {
                const uint8_t* e = li.next(&el);
                if (!e) break;
                if (kind == LASPJ_KIND_GSET) {
                    // a G-Set element that is a 2-tuple takes the bodies' OR-Set branch
                    // (lasp_core.erl:467-474, 648-655, 688-695): its first component is the
                    // fun's argument
                    uint32_t slot = 0;
                    if ((st = reg_elem(d, e, el, &slot))) break;
                    it->keys.push_back(slot);
                    it->toff.push_back((uint32_t)it->toks.size());
                    continue;
                }
                // {Key, [{Token, Bool}, ...]}
                if (el < 2 || e[0] != kSmallTuple || e[1] != 2) { st = LASPJ_DEC_MALFORMED; break; }
                const size_t kl = term_len(e + 2, el - 2);
                if (!kl) { st = LASPJ_DEC_MALFORMED; break; }
                uint32_t key = 0;
                if ((st = reg_elem(d, e + 2, kl, &key))) break;
                const uint8_t* c = e + 2 + kl;
                const size_t cl = el - 2 - kl;
                if (c[0] != kNil && c[0] != kList) { st = LASPJ_DEC_MALFORMED; break; }
                if (c[0] == kList) {
                    ListIt ci(c, cl);
                    size_t rl;
                    while (const uint8_t* r = ci.next(&rl)) {
                        if (rl < 2 || r[0] != kSmallTuple || r[1] != 2) { st = LASPJ_DEC_MALFORMED; break; }
                        const size_t tl = term_len(r + 2, rl - 2);
                        if (!tl) { st = LASPJ_DEC_MALFORMED; break; }
                        const int flag = bool_atom(r + 2 + tl);
                        if (flag < 0 || term_len(r + 2 + tl, rl - 2 - tl) != rl - 2 - tl) {
                            st = LASPJ_DEC_MALFORMED;
                            break;
                        }
                        uint16_t ts = 0;
                        if ((st = reg_tok(d, key, r + 2, tl, &ts))) break;
                        it->toks.push_back((64ull * key + ts) | (flag ? kFlagBit : 0ull));
                    }
                    if (st == LASPJ_DEC_OK && ci.tail() && ci.tail()[0] != kNil) st = LASPJ_DEC_MALFORMED;
                }
                if (st) break;
                it->keys.push_back(key);
                it->toff.push_back((uint32_t)it->toks.size());
            }
            if (st == LASPJ_DEC_OK && li.tail() && li.tail()[0] != kNil) st = LASPJ_DEC_MALFORMED;
        }
        if (st == LASPJ_DEC_OK && args) {
            // the fun's argument per entry: the key (OR-Set), the element or the first
            // component of a 2-tuple element (G-Set), as slots of the dictionary
            args->clear();
            for (uint64_t k : it->keys) {
                const uint32_t e = (uint32_t)k;
                std::string_view img = d->elems[e];
                uint32_t a = e;
                if (kind == LASPJ_KIND_GSET && img.size() >= 2 && (uint8_t)img[0] == kSmallTuple &&
                    (uint8_t)img[1] == 2) {
                    const size_t l0 = term_len((const uint8_t*)img.data() + 2, img.size() - 2);
                    if ((st = reg_elem(d, (const uint8_t*)img.data() + 2, l0, &a))) break;
                }
                args->push_back(a);
            }
        }
    } catch (const std::bad_alloc&) {
        d->rollback();
        d->journal.clear();
        return LASPJ_E_NOMEM;
    }
    if (st != LASPJ_DEC_OK) d->rollback();
    d->journal.clear();
    return st;
}

int list_register(laspj_dict* dict, const uint8_t* img, size_t n, uint32_t* slot) {
    Dict* d = &dict->d;
    d->journal.clear();
    int st;
    try {
        if (term_len(img, n) != n) return LASPJ_DEC_MALFORMED;
        st = reg_elem(d, img, n, slot);
    } catch (const std::bad_alloc&) {
        d->rollback();
        d->journal.clear();
        return LASPJ_E_NOMEM;
    }
    if (st) d->rollback();
    d->journal.clear();
    return st;
}

std::string_view list_elem_image(const laspj_dict* dict, uint32_t e) {
    return dict->d.elems[e];
}

std::string_view list_tok_image(const laspj_dict* dict, uint64_t g) {
    return dict->d.toks[(size_t)(g >> 6)][(size_t)(g & 63)];
}

size_t list_term_len(const uint8_t* p, size_t n) { return term_len(p, n); }

// dense ranks in term order: krank per element slot, grank per token g = 64 e + k (equal
// terms share a rank; tokens of different elements are ordered together)
int list_ranks(const laspj_dict* dict, std::vector<uint32_t>* krank, std::vector<uint32_t>* grank) {
    const Dict& d = dict->d;
    const uint32_t K = (uint32_t)d.elems.size();
    try {
        std::vector<uint32_t> o(K);
        for (uint32_t e = 0; e < K; ++e) o[e] = e;
        std::stable_sort(o.begin(), o.end(), [&](uint32_t x, uint32_t y) {
            return cmp_view(d.elems[x], d.elems[y]) < 0;
        });
        krank->assign(K, 0);
        uint32_t r = 0;
        for (uint32_t i = 0; i < K; ++i) {
            if (i && cmp_view(d.elems[o[i - 1]], d.elems[o[i]]) != 0) ++r;
            (*krank)[o[i]] = r;
        }
        std::vector<uint64_t> g;
        for (uint32_t e = 0; e < K; ++e)
            for (uint32_t k = 0; k < d.toks[e].size(); ++k) g.push_back(64ull * e + k);
        auto img = [&](uint64_t x) { return d.toks[(size_t)(x >> 6)][(size_t)(x & 63)]; };
        std::stable_sort(g.begin(), g.end(), [&](uint64_t x, uint64_t y) {
            return cmp_view(img(x), img(y)) < 0;
        });
        grank->assign(64ull * std::max<uint32_t>(K, 1), 0);
        r = 0;
        for (size_t i = 0; i < g.size(); ++i) {
            if (i && cmp_view(img(g[i - 1]), img(g[i])) != 0) ++r;
            (*grank)[g[i]] = r;
        }
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
    return LASPJ_OK;
}

// items -> term_to_binary image (131 + the list), as term_to_binary/1 writes it: LIST_EXT
// (STRING_EXT for a G-Set list of integers 0..255, NIL_EXT when empty), {Key, Tokens}
// 2-tuples, pair keys {X, Y}, pair tokens [Tx, Ty], flags as ATOM_EXT
int list_write(const laspj_dict* dict, int32_t kind, const ListItems& it, std::string* out) {
    const Dict& d = dict->d;
    try {
        out->clear();
        out->push_back((char)131);
        const size_t n = it.keys.size();
        if (n == 0) {
            out->push_back((char)kNil);
            return LASPJ_OK;
        }
        auto key_img = [&](uint64_t k, std::string* o) {
            if (k & kPairBit) {
                o->push_back((char)kSmallTuple);
                o->push_back(2);
                o->append(d.elems[(size_t)((k >> 31) & 0x7FFFFFFFull)]);
                o->append(d.elems[(size_t)(k & 0x7FFFFFFFull)]);
            } else {
                o->append(d.elems[(size_t)(k & 0x7FFFFFFFull)]);
            }
        };
        auto tok = [&](uint64_t g) { return d.toks[(size_t)(g >> 6)][(size_t)(g & 63)]; };
        if (kind == LASPJ_KIND_GSET) {
            bool bytes = n < 65536;
            std::vector<uint8_t> b;
            for (size_t i = 0; bytes && i < n; ++i) {
                uint8_t v;
                bytes = !(it.keys[i] & kPairBit) && small_int(d.elems[(size_t)it.keys[i]], &v);
                b.push_back(v);
            }
            if (bytes) {
                out->push_back((char)kString);
                out->push_back((char)((n >> 8) & 0xFF));
                out->push_back((char)(n & 0xFF));
                out->append((const char*)b.data(), n);
                return LASPJ_OK;
            }
            out->push_back((char)kList);
            put_be32(out, (uint32_t)n);
            for (size_t i = 0; i < n; ++i) key_img(it.keys[i], out);
            out->push_back((char)kNil);
            return LASPJ_OK;
        }
        out->push_back((char)kList);
        put_be32(out, (uint32_t)n);
        for (size_t i = 0; i < n; ++i) {
            out->push_back((char)kSmallTuple);
            out->push_back(2);
            key_img(it.keys[i], out);
            const uint32_t a = it.toff[i], b = it.toff[i + 1];
            if (a == b) {
                out->push_back((char)kNil);
                continue;
            }
            out->push_back((char)kList);
            put_be32(out, b - a);
            for (uint32_t j = a; j < b; ++j) {
                const uint64_t t = it.toks[j];
                out->push_back((char)kSmallTuple);
                out->push_back(2);
                if (t & kPairBit) {
                    std::string_view x = tok((t >> 31) & 0x7FFFFFFFull), y = tok(t & 0x7FFFFFFFull);
                    uint8_t vx, vy;
                    if (small_int(x, &vx) && small_int(y, &vy)) {
                        out->push_back((char)kString);
                        out->push_back(0);
                        out->push_back(2);
                        out->push_back((char)vx);
                        out->push_back((char)vy);
                    } else {
                        out->push_back((char)kList);
                        put_be32(out, 2);
                        out->append(x);
                        out->append(y);
                        out->push_back((char)kNil);
                    }
                } else {
                    out->append(tok(t & 0x7FFFFFFFull));
                }
                static const char kTrue[7] = {100, 0, 4, 't', 'r', 'u', 'e'};
                static const char kFalse[8] = {100, 0, 5, 'f', 'a', 'l', 's', 'e'};
                if (t & kFlagBit) out->append(kTrue, 7);
                else out->append(kFalse, 8);
            }
            out->push_back((char)kNil);
        }
        out->push_back((char)kNil);
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
    return LASPJ_OK;
}

uint32_t list_dict_elements(const laspj_dict* dict) { return (uint32_t)dict->d.elems.size(); }

// ------------------------------------------------------------------ update/3 operations
// (laspj_nif.hip's laspj_var_etf_update): the Op term of Type:update(Op, Actor, Value0)
// read from its image, then its element / token terms registered one by one.

namespace {

// `a` is the atom image of `name` (any of the four atom encodings)
bool is_atom(const uint8_t* a, size_t n, const char* name) {
    if (!n || term_class(a[0]) != 1 || term_len(a, n) != n) return false;
    return atom_name(a) == name;
}

struct OpParser {
    int32_t kind;
    std::vector<UpdateOp>* out;
    int depth = 0;

    // the elements of a proper list image (LIST_EXT / STRING_EXT / NIL_EXT) in order
    template <class F>
    bool each(const uint8_t* l, size_t n, F f) {
        if (!n) return false;
        if (l[0] == kNil) return n == 1;
        if ((l[0] != kList && l[0] != kString) || term_len(l, n) != n) return false;
        ListIt it(l, n);
        size_t el;
        while (const uint8_t* e = it.next(&el))
            if (!el || !f(e, el)) return false;
        return !it.tail() || it.tail()[0] == kNil;
    }

    void push(uint8_t k, const uint8_t* e, size_t el, const uint8_t* t, size_t tl) {
        UpdateOp o;
        o.kind = k;
        o.elem.assign((const char*)e, el);
        if (t) o.tok.assign((const char*)t, tl);
        o.mint = k == LASPJ_OP_ADD && kind == LASPJ_KIND_ORSET && !t;
        out->push_back(std::move(o));
    }

    // one operation (lasp_orset.erl:101-117 / lasp_gset.erl:84-88); false: no clause of
    // the reference's update/3 takes it as written (function_clause, a badmatch inside
    // add_all's fold, a crash in remove_elems / apply_ops over an improper list ...)
    bool op(const uint8_t* p, size_t n) {
        if (++depth > 64) return false;
        if (n < 2 || (p[0] != kSmallTuple && p[0] != kLargeTuple) || term_len(p, n) != n)
            return false;
        const uint64_t ar = p[0] == kSmallTuple ? p[1] : be32(p + 1);
        size_t off = p[0] == kSmallTuple ? 2 : 5;
        const uint8_t* f[3];
        size_t fl[3];
        if (ar < 2 || ar > 3) return false;
        for (uint64_t i = 0; i < ar; ++i) {
            f[i] = p + off;
            fl[i] = term_len(p + off, n - off);
            if (!fl[i]) return false;
            off += fl[i];
        }
        const bool orset = kind == LASPJ_KIND_ORSET;
        if (ar == 3)
            return orset && is_atom(f[0], fl[0], "add_by_token") &&
                   (push(LASPJ_OP_ADD, f[2], fl[2], f[1], fl[1]), true);
        if (is_atom(f[0], fl[0], "add")) {
            push(LASPJ_OP_ADD, f[1], fl[1], nullptr, 0);
            return true;
        }
        if (is_atom(f[0], fl[0], "add_all"))
            return each(f[1], fl[1], [&](const uint8_t* e, size_t el) {
                push(LASPJ_OP_ADD, e, el, nullptr, 0);
                return true;
            });
        if (!orset) return false;
        if (is_atom(f[0], fl[0], "remove")) {
            push(LASPJ_OP_REMOVE, f[1], fl[1], nullptr, 0);
            return true;
        }
        if (is_atom(f[0], fl[0], "remove_all"))
            return each(f[1], fl[1], [&](const uint8_t* e, size_t el) {
                push(LASPJ_OP_REMOVE, e, el, nullptr, 0);
                return true;
            });
        if (is_atom(f[0], fl[0], "update"))
            return each(f[1], fl[1], [&](const uint8_t* e, size_t el) { return op(e, el); });
        return false;
    }
};

}  // namespace

int parse_update_op(int32_t kind, const uint8_t* img, size_t n, std::vector<UpdateOp>* ops) {
    ops->clear();
    try {
        const uint8_t* t;
        size_t tn;
        if (payload_term(img, n, -1, -1, &t, &tn) != LASPJ_DEC_OK) return LASPJ_DEC_MALFORMED;
        OpParser ps{kind, ops};
        if (!ps.op(t, tn)) return LASPJ_DEC_MALFORMED;
        // every term must be one the comparator handles (the dictionary's rule)
        for (const UpdateOp& o : *ops) {
            bool ok = true;
            const auto* e = (const uint8_t*)o.elem.data();
            term_cmp(e, o.elem.size(), e, o.elem.size(), &ok);
            if (ok && !o.tok.empty()) {
                const auto* k = (const uint8_t*)o.tok.data();
                term_cmp(k, o.tok.size(), k, o.tok.size(), &ok);
            }
            if (!ok) return LASPJ_DEC_MALFORMED;
        }
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
    return LASPJ_DEC_OK;
}

int64_t dict_find_elem(const laspj_dict* dict, const uint8_t* img, size_t n) {
    const int64_t f = dict->d.elem(img, n);
    if (f >= 0) return f;
    // orddict:find/2 matches keys with `==`: another image of an equal term is not "absent"
    Dict* d = const_cast<Dict*>(&dict->d);
    uint64_t he = 0;
    if (!eq_hash(d, img, n, kElemSeed, &he)) return -2;
    const bool eq = d->elem_eq.find_if(he, 0, [&](std::string_view o) {
        bool ok = true;
        return term_cmp(img, n, (const uint8_t*)o.data(), o.size(), &ok) == 0 && ok;
    }) != nullptr;
    return eq ? -2 : -1;
}

void dict_begin(laspj_dict* dict) { dict->d.journal.clear(); }

void dict_rollback(laspj_dict* dict) {
    dict->d.rollback();
    dict->d.journal.clear();
}

int dict_reg_elem(laspj_dict* dict, const uint8_t* img, size_t n, uint32_t* slot) {
    try {
        return reg_elem(&dict->d, img, n, slot);
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
}

bool dict_set_tok_cap(laspj_dict* dict, uint32_t cap, uint32_t max_len) {
    Dict& d = dict->d;
    if (max_len) {
        // every token registered so far of one length, at most max_len
        uint32_t tl = 0;
        for (const auto& tv : d.toks)
            for (std::string_view t : tv) {
                if (t.size() > max_len || (tl && t.size() != tl)) return false;
                tl = (uint32_t)t.size();
            }
        d.tok_len = tl;
    }
    d.tok_len_max = max_len;
    d.tok_cap = cap;
    return true;
}
uint32_t dict_tok_cap(const laspj_dict* dict) { return dict->d.tok_cap; }

int dict_export_wide(const laspj_dict* dict, WideExport* x) {
    const Dict& d = dict->d;
    const uint32_t K = (uint32_t)d.elems.size();
    try {
        x->eoff.assign(K + 1ull, 0);
        x->eblob.clear();
        for (uint32_t e = 0; e < K; ++e) {
            x->eblob.insert(x->eblob.end(), d.elems[e].begin(), d.elems[e].end());
            x->eoff[e + 1] = (uint32_t)x->eblob.size();
        }
        x->eorder.resize(K);
        for (uint32_t e = 0; e < K; ++e) x->eorder[e] = e;
        std::stable_sort(x->eorder.begin(), x->eorder.end(), [&](uint32_t a, uint32_t b) {
            return cmp_view(d.elems[a], d.elems[b]) < 0;
        });
        // tokens by element slot, each element's in term order (rank), CSR
        x->rb.assign(K + 1ull, 0);
        x->rslot.clear();
        x->tblob.clear();
        x->toff.assign(1, 0);
        x->max_cnt = 0;
        std::vector<uint16_t> ord;
        for (uint32_t e = 0; e < K; ++e) {
            const auto& tv = d.toks[e];
            ord.resize(tv.size());
            for (size_t k = 0; k < ord.size(); ++k) ord[k] = (uint16_t)k;
            std::stable_sort(ord.begin(), ord.end(), [&](uint16_t a, uint16_t b) {
                return cmp_view(tv[a], tv[b]) < 0;
            });
            for (uint16_t k : ord) {
                x->rslot.push_back(k);
                x->tblob.insert(x->tblob.end(), tv[k].begin(), tv[k].end());
                x->toff.push_back((uint32_t)x->tblob.size());
            }
            x->rb[e + 1] = (uint32_t)x->rslot.size();
            x->max_cnt = std::max<uint32_t>(x->max_cnt, (uint32_t)tv.size());
        }
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
    return LASPJ_OK;
}

int dict_reg_tok(laspj_dict* dict, uint32_t e, const uint8_t* img, size_t n, uint32_t* slot) {
    try {
        uint16_t s = 0;
        const int st = reg_tok(&dict->d, e, img, n, &s);
        *slot = s;
        return st;
    } catch (const std::bad_alloc&) {
        return LASPJ_E_NOMEM;
    }
}

}  // namespace laspj
