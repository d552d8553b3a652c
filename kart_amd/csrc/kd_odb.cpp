// kd_odb.cpp — the git object database read natively (loose objects, pack v2 with idx v1/v2,
// zlib, OFS/REF delta chains) and Dataset3's leaf walk over it, with tree-OID pruning.
//
// Replaces what Kart gets from libgit2 (koordinates fork @ bb69c8fa, vendor/libgit2/Makefile:1-3)
// on the diff path: the feature-tree iteration of Dataset3 (kart/dataset3.py:26-35,225-231), the
// blob reads of BaseDataset.get_blob_at (kart/base_dataset.py:230-265), and the subtree pruning
// of tree-to-tree diff (pygit2 Tree.diff_to_tree, called at kart/rich_base_dataset.py:212-232):
// a subtree whose OID is the same in both trees is never opened.
//
// Host code (no GPU).  The walk feeds the packer (kd_pack_*_keys, kd_sort_side): its output is
// the flat (path arena, offsets, OIDs) layout those take.  Formats follow git's documented ones
// (Documentation/technical/pack-format.txt): idx v2 = magic, fanout[256], sha[n], crc[n],
// off32[n] (MSB -> index into off64[]); pack entries = type/size varint header, zlib stream;
// OFS_DELTA base = this offset - (offset varint); delta = src/dst size varints + copy/insert ops.
#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kartdiff.h"

namespace kd {
void set_error(const char* fmt, ...);
}

namespace {

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

enum { OBJ_COMMIT = 1, OBJ_TREE = 2, OBJ_BLOB = 3, OBJ_TAG = 4, OBJ_OFS_DELTA = 6, OBJ_REF_DELTA = 7 };
enum { RD_OK = 0, RD_MISSING = 1, RD_CORRUPT = 2 };

constexpr int MAX_CHAIN = 10000;       // delta chain guard (git's default depth is 50)
constexpr u64 CACHE_MAX_OBJ = 1 << 16; // resolved objects at most this big enter the base cache
constexpr int CACHE_SLOTS = 1024;      // per reader, direct-mapped by pack offset

inline u32 be32(const u8* p) { return (u32)p[0] << 24 | (u32)p[1] << 16 | (u32)p[2] << 8 | p[3]; }
inline u64 be64(const u8* p) { return (u64)be32(p) << 32 | be32(p + 4); }

struct MappedFile {
    const u8* p = nullptr;
    size_t n = 0;
    bool open(const std::string& path) {
        int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0 || st.st_size <= 0) { ::close(fd); return false; }
        void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        if (m == MAP_FAILED) return false;
        p = (const u8*)m;
        n = (size_t)st.st_size;
        return true;
    }
    ~MappedFile() {
        if (p) munmap((void*)p, n);
    }
};

struct Pack {
    MappedFile idx, pack;
    int ver = 0;  // idx version 1 or 2
    u32 n = 0;
    const u8 *fan = nullptr, *sha = nullptr, *off32 = nullptr, *off64 = nullptr;
    size_t n64 = 0;

    bool open(const std::string& idx_path, const std::string& pack_path) {
        if (!idx.open(idx_path) || !pack.open(pack_path)) return false;
        if (pack.n < 32 || memcmp(pack.p, "PACK", 4) != 0) return false;
        const u32 pv = be32(pack.p + 4);
        if (pv != 2 && pv != 3) return false;
        const u8* p = idx.p;
        if (idx.n >= 8 && memcmp(p, "\377tOc", 4) == 0) {
            if (be32(p + 4) != 2) return false;
            ver = 2;
            fan = p + 8;
            if (idx.n < 8 + 1024) return false;
            n = be32(fan + 4 * 255);
            const size_t need = 8 + 1024 + (size_t)n * 28 + 40;
            if (idx.n < need) return false;
            sha = fan + 1024;
            off32 = sha + (size_t)n * 24;  // after sha[n] and crc[n]
            off64 = off32 + (size_t)n * 4;
            n64 = (idx.n - need) / 8;
        } else {
            ver = 1;
            fan = p;
            if (idx.n < 1024) return false;
            n = be32(fan + 4 * 255);
            if (idx.n < 1024 + (size_t)n * 24 + 40) return false;
        }
        return true;
    }

    // offset of `oid` in the pack, or false
    bool find(const u8* oid, u64* off) const {
        u32 lo = oid[0] ? be32(fan + 4 * (oid[0] - 1)) : 0, hi = be32(fan + 4 * oid[0]);
        if (hi > n || lo > hi) return false;
        while (lo < hi) {
            const u32 mid = lo + (hi - lo) / 2;
            const u8* s = ver == 2 ? sha + 20 * (size_t)mid : fan + 1024 + 24 * (size_t)mid + 4;
            const int c = memcmp(s, oid, 20);
            if (c == 0) {
                if (ver == 1) { *off = be32(fan + 1024 + 24 * (size_t)mid); return true; }
                const u32 o = be32(off32 + 4 * (size_t)mid);
                if (!(o & 0x80000000u)) { *off = o; return true; }
                const size_t j = o & 0x7FFFFFFFu;
                if (j >= n64) return false;
                *off = be64(off64 + 8 * j);
                return true;
            }
            if (c < 0) lo = mid + 1;
            else hi = mid;
        }
        return false;
    }
};

}  // namespace

namespace {
struct Reader;
}

struct kd_odb {
    std::vector<std::string> objdirs;  // objects/ and its alternates
    std::vector<std::unique_ptr<Pack>> packs;
    // idle readers (zlib stream + base cache) reused by single-object reads: building one costs
    // more than reading a small object (ctypes drops the GIL, so calls may be concurrent)
    std::mutex pool_mu;
    std::vector<Reader*> pool;
    // options (kd_odb_set_option; kd_odb_open seeds them from the environment)
    int zlib_only = 0;  // "zlib" [KD_ODB_ZLIB]: 1 = inflate with zlib even when libdeflate is present (A/B)
};

namespace {

void add_objdir(kd_odb* db, const std::string& dir, int depth) {
    for (auto& d : db->objdirs)
        if (d == dir) return;
    db->objdirs.push_back(dir);
    if (DIR* dp = opendir((dir + "/pack").c_str())) {
        std::vector<std::string> names;
        while (struct dirent* e = readdir(dp)) {
            std::string nm = e->d_name;
            if (nm.size() > 4 && nm.compare(nm.size() - 4, 4, ".idx") == 0) names.push_back(nm);
        }
        closedir(dp);
        std::sort(names.begin(), names.end());
        for (auto& nm : names) {
            auto pk = std::make_unique<Pack>();
            const std::string base = dir + "/pack/" + nm.substr(0, nm.size() - 4);
            if (pk->open(base + ".idx", base + ".pack")) db->packs.push_back(std::move(pk));
        }
    }
    if (depth >= 5) return;
    FILE* f = fopen((dir + "/info/alternates").c_str(), "r");
    if (!f) return;
    char line[4096];
    while (fgets(line, sizeof line, f)) {
        std::string s = line;
        while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
        if (s.empty() || s[0] == '#') continue;
        add_objdir(db, s[0] == '/' ? s : dir + "/" + s, depth + 1);
    }
    fclose(f);
}

int read_varint_le(const u8* d, size_t n, size_t* i, u64* out) {
    u64 v = 0;
    int shift = 0;
    for (;;) {
        if (*i >= n || shift > 63) return -1;
        const u8 c = d[(*i)++];
        v |= (u64)(c & 0x7F) << shift;
        shift += 7;
        if (!(c & 0x80)) break;
    }
    *out = v;
    return 0;
}

// git's delta: src size, dst size, then ops (copy from base: 0x80 | offset/size byte masks;
// insert: 1..127 literal bytes)
int apply_delta(const u8* base, size_t blen, const u8* d, size_t dlen, std::vector<u8>& out) {
    size_t i = 0;
    u64 src, dst;
    if (read_varint_le(d, dlen, &i, &src) || read_varint_le(d, dlen, &i, &dst)) return -1;
    if (src != blen) return -1;
    out.resize(dst);
    u8* o = out.data();
    u64 w = 0;
    while (i < dlen) {
        const u8 op = d[i++];
        if (op & 0x80) {
            u64 off = 0, sz = 0;
            for (int b = 0; b < 4; b++)
                if (op & (1 << b)) {
                    if (i >= dlen) return -1;
                    off |= (u64)d[i++] << (8 * b);
                }
            for (int b = 0; b < 3; b++)
                if (op & (0x10 << b)) {
                    if (i >= dlen) return -1;
                    sz |= (u64)d[i++] << (8 * b);
                }
            if (sz == 0) sz = 0x10000;
            if (off + sz > blen || w + sz > dst) return -1;
            memcpy(o + w, base + off, sz);
            w += sz;
        } else if (op) {
            if (i + op > dlen || w + op > dst) return -1;
            memcpy(o + w, d + i, op);
            i += op;
            w += op;
        } else {
            return -1;
        }
    }
    return w == dst ? 0 : -1;
}

// libdeflate (the image's libdeflate.so.0, when present) inflates a whole zlib stream of known
// size in one call, without zlib's per-stream state machine: a pack read is mostly tiny delta
// streams, so this is most of its CPU time.  Its documented C API, declared here (no header in the
// image); zlib when the library is absent.
struct Deflate {
    typedef void* (*alloc_fn)();
    typedef void (*free_fn)(void*);
    typedef int (*zlib_ex_fn)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);
    alloc_fn alloc = nullptr;
    free_fn release = nullptr;
    zlib_ex_fn zlib_ex = nullptr;
    Deflate() {
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (alloc_fn)dlsym(h, "libdeflate_alloc_decompressor");
        release = (free_fn)dlsym(h, "libdeflate_free_decompressor");
        zlib_ex = (zlib_ex_fn)dlsym(h, "libdeflate_zlib_decompress_ex");
        if (!alloc || !release || !zlib_ex) alloc = nullptr;
    }
    bool ok() const { return alloc != nullptr; }
};
const Deflate& deflate_lib() {
    static const Deflate d;
    return d;
}

// One thread's reader: a zlib stream, a delta-base cache, scratch buffers.
struct Reader {
    const kd_odb* db;
    z_stream z;
    bool zok = false;
    struct Slot {
        const Pack* pk = nullptr;
        u64 off = ~0ull;
        int type = 0;
        std::vector<u8> data;
    };
    std::vector<Slot> cache;
    std::vector<u8> dbuf, tmp;

    void* dec = nullptr;  // libdeflate decompressor

    explicit Reader(const kd_odb* d) : db(d), cache(CACHE_SLOTS) {
        memset(&z, 0, sizeof z);
        zok = inflateInit(&z) == Z_OK;
        if (!d->zlib_only && deflate_lib().ok()) dec = deflate_lib().alloc();
    }
    ~Reader() {
        if (zok) inflateEnd(&z);
        if (dec) deflate_lib().release(dec);
    }
    Reader(const Reader&) = delete;

    // inflate one zlib stream starting at src into exactly `size` bytes
    int inflate_exact(const u8* src, size_t avail, u8* dst, size_t size) {
        if (dec) {
            u8 dummy;
            size_t in_used = 0, out_used = 0;
            const int r = deflate_lib().zlib_ex(dec, src, avail, size ? dst : &dummy, size, &in_used, &out_used);
            return r == 0 && out_used == size ? RD_OK : RD_CORRUPT;  // 0: LIBDEFLATE_SUCCESS
        }
        if (!zok || inflateReset(&z) != Z_OK) return RD_CORRUPT;
        z.next_in = (Bytef*)src;
        z.avail_in = (uInt)std::min<size_t>(avail, 0xFFFFFFFFu);
        u8 dummy;
        z.next_out = size ? dst : &dummy;
        z.avail_out = (uInt)size;
        const int r = inflate(&z, Z_FINISH);
        if (r != Z_STREAM_END || z.total_out != size) return RD_CORRUPT;
        return RD_OK;
    }

    Slot& slot(const Pack* pk, u64 off) { return cache[(off * 0x9E3779B97F4A7C15ull) >> 54 & (CACHE_SLOTS - 1)]; }

    // entry header at `off`: type, inflated size, start of the zlib data (after the delta base)
    int entry_header(const Pack& pk, u64 off, int* type, u64* size, u64* data, u64* base_off, const u8** base_oid) {
        const u8* p = pk.pack.p;
        const u64 n = pk.pack.n - 20;  // trailing checksum
        if (off < 12 || off >= n) return RD_CORRUPT;
        u64 i = off;
        u8 c = p[i++];
        *type = (c >> 4) & 7;
        u64 sz = c & 15;
        int shift = 4;
        while (c & 0x80) {
            if (i >= n || shift > 60) return RD_CORRUPT;
            c = p[i++];
            sz |= (u64)(c & 0x7F) << shift;
            shift += 7;
        }
        *size = sz;
        if (*type == OBJ_OFS_DELTA) {
            if (i >= n) return RD_CORRUPT;
            c = p[i++];
            u64 rel = c & 0x7F;
            while (c & 0x80) {
                if (i >= n || rel >= (1ull << 56)) return RD_CORRUPT;
                c = p[i++];
                rel = ((rel + 1) << 7) | (c & 0x7F);
            }
            if (rel == 0 || rel > off) return RD_CORRUPT;
            *base_off = off - rel;
        } else if (*type == OBJ_REF_DELTA) {
            if (i + 20 > n) return RD_CORRUPT;
            *base_oid = p + i;
            i += 20;
        } else if (*type < OBJ_COMMIT || *type > OBJ_TAG) {
            return RD_CORRUPT;
        }
        *data = i;
        return RD_OK;
    }

    // object at `off` of `pk` (delta chains resolved) into out
    int read_packed(const Pack& pk, u64 off, int* type, std::vector<u8>& out, int depth = 0) {
        struct Link { u64 off, data, size; };
        std::vector<Link> chain;
        u64 cur = off;
        int btype = 0;
        for (;;) {
            Slot& s = slot(&pk, cur);
            if (s.pk == &pk && s.off == cur) {  // resolved before
                out = s.data;
                btype = s.type;
                break;
            }
            int t;
            u64 sz, data, boff = 0;
            const u8* boid = nullptr;
            int rc = entry_header(pk, cur, &t, &sz, &data, &boff, &boid);
            if (rc) return rc;
            if (t == OBJ_OFS_DELTA || t == OBJ_REF_DELTA) {
                if ((int)chain.size() >= MAX_CHAIN) return RD_CORRUPT;
                chain.push_back({cur, data, sz});
                if (t == OBJ_OFS_DELTA) {
                    cur = boff;
                    continue;
                }
                u64 o;
                if (pk.find(boid, &o)) {
                    cur = o;
                    continue;
                }
                if (depth > 8) return RD_CORRUPT;
                rc = read(boid, &btype, out, depth + 1);  // base in another pack / loose (thin pack fixed up)
                if (rc) return rc == RD_MISSING ? RD_CORRUPT : rc;
                break;
            }
            out.resize(sz);
            rc = inflate_exact(pk.pack.p + data, pk.pack.n - data, out.data(), sz);
            if (rc) return rc;
            btype = t;
            // a chain's base, and every whole tree: a compare walk reads the old side's tree just
            // before the new side's, which git stores as a delta against it
            if (!chain.empty() || t == OBJ_TREE) remember(&pk, cur, t, out);
            break;
        }
        for (size_t j = chain.size(); j-- > 0;) {
            const Link& L = chain[j];
            dbuf.resize(L.size);
            int rc = inflate_exact(pk.pack.p + L.data, pk.pack.n - L.data, dbuf.data(), L.size);
            if (rc) return rc;
            if (apply_delta(out.data(), out.size(), dbuf.data(), dbuf.size(), tmp)) return RD_CORRUPT;
            out.swap(tmp);
            // every resolved link, the object itself included: in a batch read in pack order the
            // next object is usually a delta against this one (fast-import and repack chains)
            remember(&pk, L.off, btype, out);
        }
        *type = btype;
        return RD_OK;
    }

    void remember(const Pack* pk, u64 off, int type, const std::vector<u8>& data) {
        if (data.size() > CACHE_MAX_OBJ) return;
        Slot& s = slot(pk, off);
        s.pk = pk;
        s.off = off;
        s.type = type;
        s.data = data;
    }

    // one loose object file: zlib("<type> <size>\0" + content)
    int parse_loose(const std::vector<u8>& raw, int* type, std::vector<u8>& out) {
        if (!zok || inflateReset(&z) != Z_OK) return RD_CORRUPT;
        u8 hdr[64];
        z.next_in = const_cast<u8*>(raw.data());
        z.avail_in = (uInt)raw.size();
        z.next_out = hdr;
        z.avail_out = sizeof hdr;
        int zr = inflate(&z, Z_NO_FLUSH);
        if (zr != Z_OK && zr != Z_STREAM_END) return RD_CORRUPT;
        const size_t got = sizeof hdr - z.avail_out;
        const u8* nul = (const u8*)memchr(hdr, 0, got);
        if (!nul) return RD_CORRUPT;
        const u8* sp = (const u8*)memchr(hdr, ' ', nul - hdr);
        if (!sp) return RD_CORRUPT;
        const size_t tl = sp - hdr;
        int t = tl == 4 && !memcmp(hdr, "blob", 4) ? OBJ_BLOB
                : tl == 4 && !memcmp(hdr, "tree", 4) ? OBJ_TREE
                : tl == 6 && !memcmp(hdr, "commit", 6) ? OBJ_COMMIT
                : tl == 3 && !memcmp(hdr, "tag", 3) ? OBJ_TAG : 0;
        if (!t) return RD_CORRUPT;
        u64 size = 0;
        for (const u8* q = sp + 1; q < nul; q++) {
            if (*q < '0' || *q > '9' || size > (1ull << 50)) return RD_CORRUPT;
            size = size * 10 + (*q - '0');
        }
        const size_t have = got - (nul + 1 - hdr);
        if (have > size) return RD_CORRUPT;
        out.resize(size);
        memcpy(out.data(), nul + 1, have);
        if (zr != Z_STREAM_END) {
            z.next_out = out.data() + have;
            z.avail_out = (uInt)(size - have);
            zr = inflate(&z, Z_FINISH);
            if (zr != Z_STREAM_END) return RD_CORRUPT;
        }
        if (z.total_out != size + (nul + 1 - hdr)) return RD_CORRUPT;
        *type = t;
        return RD_OK;
    }

    // the object's loose file in the first object directory (own, then alternates) that holds a
    // readable copy: a corrupt copy in one directory does not hide a good one in the next
    int read_loose(const u8* oid, int* type, std::vector<u8>& out) {
        static const char hx[] = "0123456789abcdef";
        char name[42];
        for (int i = 0; i < 20; i++) {
            name[2 * i] = hx[oid[i] >> 4];
            name[2 * i + 1] = hx[oid[i] & 15];
        }
        int result = RD_MISSING;
        for (const std::string& dir : db->objdirs) {
            std::string path = dir + "/" + std::string(name, 2) + "/" + std::string(name + 2, 38);
            int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
            if (fd < 0) continue;
            std::vector<u8> raw;
            u8 buf[65536];
            ssize_t r;
            while ((r = ::read(fd, buf, sizeof buf)) > 0) raw.insert(raw.end(), buf, buf + r);
            ::close(fd);
            const int rc = r < 0 ? RD_CORRUPT : parse_loose(raw, type, out);
            if (rc == RD_OK) return RD_OK;
            result = rc;
        }
        return result;
    }

    // the pack holding oid, or -1.  The packs that held the last few objects are searched first,
    // most recent first: a batch's objects tend to share packs, a compare walk alternates between
    // its roots' packs (one per side and subtree in a repository written by parallel imports), and
    // every miss is a binary search of another index
    static constexpr int MRU = 4;
    size_t mru[MRU] = {~size_t(0), ~size_t(0), ~size_t(0), ~size_t(0)};
    long locate(const u8* oid, u64* off) {
        const size_t np = db->packs.size();
        for (int j = 0; j < MRU; j++) {
            const size_t p = mru[j];
            if (p >= np) break;
            if (db->packs[p]->find(oid, off)) {
                for (int q = j; q > 0; q--) mru[q] = mru[q - 1];
                mru[0] = p;
                return (long)p;
            }
        }
        for (size_t p = 0; p < np; p++) {
            bool tried = false;
            for (int j = 0; j < MRU; j++) tried |= mru[j] == p;
            if (tried || !db->packs[p]->find(oid, off)) continue;
            for (int q = MRU - 1; q > 0; q--) mru[q] = mru[q - 1];
            mru[0] = p;
            return (long)p;
        }
        return -1;
    }

    int read(const u8* oid, int* type, std::vector<u8>& out, int depth = 0) {
        u64 off;
        const long p = locate(oid, &off);
        if (p >= 0) return read_packed(*db->packs[p], off, type, out, depth);
        return read_loose(oid, type, out);
    }
};

void hex40(const u8* oid, char* out) {
    static const char hx[] = "0123456789abcdef";
    for (int i = 0; i < 20; i++) {
        out[2 * i] = hx[oid[i] >> 4];
        out[2 * i + 1] = hx[oid[i] & 15];
    }
    out[40] = 0;
}

bool unhex40(const u8* s, u8* oid) {
    for (int i = 0; i < 20; i++) {
        int v = 0;
        for (int j = 0; j < 2; j++) {
            const u8 c = s[2 * i + j];
            const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
            if (d < 0) return false;
            v = v * 16 + d;
        }
        oid[i] = (u8)v;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// trees
// ---------------------------------------------------------------------------------------------
struct TEnt {
    const u8* name;
    u32 nlen;
    u32 mode;
    const u8* oid;
    bool tree() const { return mode == 040000; }
};

bool parse_tree(const std::vector<u8>& t, std::vector<TEnt>& out) {
    out.clear();
    const u8 *p = t.data(), *end = p + t.size();
    while (p < end) {
        u32 mode = 0;
        while (p < end && *p != ' ') {
            if (*p < '0' || *p > '7') return false;
            mode = mode * 8 + (*p++ - '0');
        }
        if (p >= end) return false;
        const u8* name = ++p;
        const u8* nul = (const u8*)memchr(p, 0, end - p);
        if (!nul || nul == name || nul + 21 > end) return false;
        out.push_back({name, (u32)(nul - name), mode, nul + 1});
        p = nul + 21;
    }
    return true;
}

// git's tree order: names compared bytewise, a tree's name continuing with '/'
int git_cmp(const TEnt& a, const TEnt& b) {
    const u32 n = std::min(a.nlen, b.nlen);
    const int c = memcmp(a.name, b.name, n);
    if (c) return c;
    const int ca = n < a.nlen ? a.name[n] : (a.tree() ? '/' : 0);
    const int cb = n < b.nlen ? b.name[n] : (b.tree() ? '/' : 0);
    return ca - cb;
}

constexpr int KMAX = 3;

struct WalkOut {
    std::string path;
    std::vector<u64> end;  // end offset of each path in `path`
    std::vector<u8> oid;
    std::vector<u32> mode;
    void add(const std::string& p, const u8* o, u32 m) {
        path += p;
        end.push_back(path.size());
        oid.insert(oid.end(), o, o + 20);
        mode.push_back(m);
    }
};

// a walk item: one path with its entry in each root (a leaf group or a subtree group)
struct Item {
    std::string path;  // relative to the walked tree
    bool tree = false;
    u8 has[KMAX] = {0, 0, 0};
    u8 oid[KMAX][20];
    u32 mode[KMAX] = {0, 0, 0};
};

struct Walk {
    int k, c0, c1;
    std::atomic<int> err{0};
    std::mutex emu;
    std::string emsg;
    void fail(int code, const std::string& m) {
        int z = 0;
        if (err.compare_exchange_strong(z, code)) {
            std::lock_guard<std::mutex> g(emu);
            emsg = m;
        }
    }

    // pruned?  (entries identical in the two compared roots; absent in both counts as identical)
    bool pruned(const Item& it) const {
        if (c0 < 0) return false;
        if (it.has[c0] != it.has[c1]) return false;
        if (!it.has[c0]) return true;
        return it.mode[c0] == it.mode[c1] && !memcmp(it.oid[c0], it.oid[c1], 20);
    }
    bool pruned(const TEnt* const* e) const {
        if (c0 < 0) return false;
        const TEnt *x = e[c0], *y = e[c1];
        if (!x || !y) return x == y;
        return x->mode == y->mode && !memcmp(x->oid, y->oid, 20);
    }

    // one level's trees of every root, parsed (a frame of the depth-first walk)
    struct Frame {
        std::vector<u8> buf[KMAX];
        std::vector<TEnt> ents[KMAX];
    };

    bool load(Reader& rd, const Item& it, Frame& f) {
        for (int r = 0; r < k && r < KMAX; r++) {
            f.ents[r].clear();
            if (!it.has[r]) continue;
            int type = 0;
            const int rc = rd.read(it.oid[r], &type, f.buf[r]);
            if (rc || type != OBJ_TREE || !parse_tree(f.buf[r], f.ents[r])) {
                char hx[41];
                hex40(it.oid[r], hx);
                if (rc) fail(rc == RD_MISSING ? KD_ENOTFOUND : KD_EINVAL,
                             std::string(rc == RD_MISSING ? "tree missing: " : "corrupt object: ") + hx);
                else fail(KD_EINVAL, std::string("not a valid tree: ") + hx);
                return false;
            }
        }
        return true;
    }

    // merge-join a frame's entries in git order: fn(e[KMAX]) per name (nullptr = absent in that
    // root), entries identical in the compared roots skipped
    template <class F>
    void join(Frame& f, F&& fn) {
        size_t pos[KMAX] = {0, 0, 0};
        for (;;) {
            int lo = -1;
            for (int r = 0; r < k && r < KMAX; r++)
                if (pos[r] < f.ents[r].size() && (lo < 0 || git_cmp(f.ents[r][pos[r]], f.ents[lo][pos[lo]]) < 0)) lo = r;
            if (lo < 0) break;
            const TEnt& e0 = f.ents[lo][pos[lo]];
            const TEnt* e[KMAX] = {nullptr, nullptr, nullptr};
            for (int r = 0; r < k && r < KMAX; r++)
                if (r == lo || (pos[r] < f.ents[r].size() && git_cmp(f.ents[r][pos[r]], e0) == 0)) e[r] = &f.ents[r][pos[r]];
            for (int r = 0; r < k && r < KMAX; r++)
                if (e[r]) pos[r]++;
            if (!pruned(e)) fn(e);
        }
    }

    Item child(const std::string& parent, const TEnt* const* e) const {
        Item c;
        const TEnt* e0 = nullptr;
        for (int r = 0; r < k && r < KMAX; r++)
            if (e[r]) {
                e0 = e0 ? e0 : e[r];
                c.has[r] = 1;
                c.mode[r] = e[r]->mode;
                memcpy(c.oid[r], e[r]->oid, 20);
            }
        c.tree = e0->tree();
        c.path = parent;
        if (!c.path.empty()) c.path += '/';
        c.path.append((const char*)e0->name, e0->nlen);
        return c;
    }

    // the children of a subtree item (breadth-first expansion of the top levels)
    template <class F>
    bool expand(Reader& rd, const Item& it, F&& fn) {
        Frame f;
        if (!load(rd, it, f)) return false;
        join(f, [&](const TEnt* const* e) { fn(child(it.path, e)); });
        return true;
    }

    // every leaf under a subtree item, depth first in git order; `path` = the item's path, grown
    // and shrunk in place, frames reused per depth (no allocation per entry)
    void descend(Reader& rd, const Item& it, std::string& path, std::vector<std::unique_ptr<Frame>>& frames,
                 WalkOut* out, int depth) {
        if (err.load(std::memory_order_relaxed)) return;
        if (depth > 64) {
            fail(KD_EINVAL, "tree nesting deeper than 64 at '" + path + "'");
            return;
        }
        if ((int)frames.size() <= depth) frames.push_back(std::make_unique<Frame>());
        Frame& f = *frames[depth];
        if (!load(rd, it, f)) return;
        const size_t plen = path.size();
        join(f, [&](const TEnt* const* e) {
            const TEnt* e0 = nullptr;
            for (int r = 0; r < k && r < KMAX && !e0; r++) e0 = e[r];
            if (e0->tree()) {
                Item c;
                for (int r = 0; r < k && r < KMAX; r++)
                    if (e[r]) {
                        c.has[r] = 1;
                        c.mode[r] = e[r]->mode;
                        memcpy(c.oid[r], e[r]->oid, 20);
                    }
                c.tree = true;
                if (plen) path += '/';
                path.append((const char*)e0->name, e0->nlen);
                descend(rd, c, path, frames, out, depth + 1);
                path.resize(plen);
                return;
            }
            for (int r = 0; r < k && r < KMAX; r++) {
                if (!e[r]) continue;
                WalkOut& o = out[r];
                o.path += path;
                if (plen) o.path += '/';
                o.path.append((const char*)e0->name, e0->nlen);
                o.end.push_back(o.path.size());
                o.oid.insert(o.oid.end(), e[r]->oid, e[r]->oid + 20);
                o.mode.push_back(e[r]->mode);
            }
        });
    }

    void walk_item(Reader& rd, const Item& it, WalkOut* out) {
        std::vector<std::unique_ptr<Frame>> frames;
        std::string path = it.path;
        descend(rd, it, path, frames, out, 0);
    }

    void emit(const Item& c, WalkOut* out) {
        for (int r = 0; r < k && r < KMAX; r++)
            if (c.has[r]) out[r].add(c.path, c.oid[r], c.mode[r]);
    }
};

template <class F>
void par_items(size_t n, int threads, F&& fn) {
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, n));
    std::atomic<size_t> next{0};
    auto work = [&](int tid) {
        for (;;) {
            const size_t i = next.fetch_add(1);
            if (i >= n) break;
            fn(i, tid);
        }
    };
    if (nt == 1) { work(0); return; }
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
}

int default_threads(int threads) {
    if (threads > 0) return std::min(threads, 256);
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}

// commit -> its tree; tree -> itself (the walk's roots may be either)
int peel_to_tree(Reader& rd, const u8* oid, u8* tree, std::string& msg) {
    std::vector<u8> buf;
    u8 cur[20];
    memcpy(cur, oid, 20);
    for (int hop = 0; hop < 8; hop++) {
        int type = 0;
        const int rc = rd.read(cur, &type, buf);
        char hx[41];
        hex40(cur, hx);
        if (rc) {
            msg = std::string(rc == RD_MISSING ? "object missing: " : "corrupt object: ") + hx;
            return rc == RD_MISSING ? KD_ENOTFOUND : KD_EINVAL;
        }
        if (type == OBJ_TREE) { memcpy(tree, cur, 20); return KD_OK; }
        const char* tag = type == OBJ_COMMIT ? "tree " : type == OBJ_TAG ? "object " : nullptr;
        const size_t tl = tag ? strlen(tag) : 0;
        if (!tag || buf.size() < tl + 40 || memcmp(buf.data(), tag, tl) != 0 || !unhex40(buf.data() + tl, cur)) {
            msg = std::string("not a tree-ish: ") + hx;
            return KD_EINVAL;
        }
    }
    msg = "tag chain too long";
    return KD_EINVAL;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
extern "C" int kd_odb_open(const char* gitdir, kd_odb** out) {
    if (!gitdir || !out) { kd::set_error("kd_odb_open: NULL"); return KD_EINVAL; }
    *out = nullptr;
    std::string dir = gitdir;
    while (dir.size() > 1 && dir.back() == '/') dir.pop_back();
    struct stat st;
    if (stat((dir + "/objects").c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) {
        kd::set_error("kd_odb_open: %s has no objects/ directory", gitdir);
        return KD_EINVAL;
    }
    kd_odb* db = new kd_odb();
    if (const char* v = std::getenv("KD_ODB_ZLIB")) db->zlib_only = (int)strtol(v, nullptr, 10) != 0;
    add_objdir(db, dir + "/objects", 0);
    *out = db;
    return KD_OK;
}

extern "C" int kd_odb_set_option(kd_odb* odb, const char* name, int64_t value) {
    if (!odb || !name) { kd::set_error("kd_odb_set_option: NULL"); return KD_EINVAL; }
    if (strcmp(name, "zlib") != 0) { kd::set_error("kd_odb_set_option: unknown option '%s'", name); return KD_EINVAL; }
    std::lock_guard<std::mutex> lk(odb->pool_mu);
    odb->zlib_only = value != 0;
    for (Reader* r : odb->pool) delete r;  // pooled readers were built for the old setting
    odb->pool.clear();
    return KD_OK;
}

extern "C" int kd_odb_get_option(kd_odb* odb, const char* name, int64_t* value) {
    if (!odb || !name || !value) { kd::set_error("kd_odb_get_option: NULL"); return KD_EINVAL; }
    if (strcmp(name, "zlib") != 0) { kd::set_error("kd_odb_get_option: unknown option '%s'", name); return KD_EINVAL; }
    *value = odb->zlib_only;
    return KD_OK;
}

extern "C" int kd_odb_close(kd_odb* odb) {
    if (odb)
        for (Reader* r : odb->pool) delete r;
    delete odb;
    return KD_OK;
}

namespace {
// a pooled reader for the duration of one call
struct PooledReader {
    kd_odb* db;
    Reader* r;
    explicit PooledReader(kd_odb* d) : db(d), r(nullptr) {
        {
            std::lock_guard<std::mutex> g(db->pool_mu);
            if (!db->pool.empty()) {
                r = db->pool.back();
                db->pool.pop_back();
            }
        }
        if (!r) r = new Reader(db);
    }
    ~PooledReader() {
        std::lock_guard<std::mutex> g(db->pool_mu);
        if (db->pool.size() < 64) db->pool.push_back(r);
        else delete r;
    }
};
}  // namespace

extern "C" int kd_odb_read(kd_odb* odb, const uint8_t* oid, int* type, uint8_t** data, uint64_t* len) {
    if (!odb || !oid || !type || !data || !len) { kd::set_error("kd_odb_read: NULL"); return KD_EINVAL; }
    *data = nullptr;
    *len = 0;
    PooledReader pr(odb);
    std::vector<u8> buf;
    const int rc = pr.r->read(oid, type, buf);
    char hx[41];
    hex40(oid, hx);
    if (rc == RD_MISSING) { kd::set_error("object %s missing", hx); return KD_ENOTFOUND; }
    if (rc) { kd::set_error("object %s corrupt", hx); return KD_EINVAL; }
    u8* p = (u8*)std::malloc(std::max<size_t>(buf.size(), 1));
    if (!p) { kd::set_error("kd_odb_read: out of memory"); return KD_EINVAL; }
    memcpy(p, buf.data(), buf.size());
    *data = p;
    *len = buf.size();
    return KD_OK;
}

extern "C" int kd_odb_read_batch(kd_odb* odb, const uint8_t* oids, uint64_t n, int threads, uint8_t** data,
                                 uint64_t* off, uint8_t* status) {
    if (!odb || !off || (n && (!oids || !status)) || !data) { kd::set_error("kd_odb_read_batch: NULL"); return KD_EINVAL; }
    *data = nullptr;
    const int nt = default_threads(threads);
    constexpr u64 CH = 256;
    const u64 nch = (n + CH - 1) / CH;
    // the objects are read in pack order (pack, then offset; loose objects last), as git's
    // unordered batch reads do: a delta chain's objects lie together (fast-import deltas each blob
    // against the one before), so the next object's base is usually in the reader's cache and a
    // chain of d deltas costs one inflate per object instead of up to d
    std::vector<std::pair<u64, u64>> ord(n);  // (pack << 48 | offset, or ~0: read by id; input index)
    std::vector<std::unique_ptr<Reader>> rds(nt);
    par_items(nch, nt, [&](size_t c, int tid) {
        if (!rds[tid]) rds[tid] = std::make_unique<Reader>(odb);
        Reader& rd = *rds[tid];
        for (u64 i = c * CH; i < std::min(n, (c + 1) * CH); i++) {
            u64 o;
            const long p = rd.locate(oids + 20 * i, &o);
            ord[i] = {p >= 0 && p < 0xFFFF && o < (1ull << 48) ? (u64)p << 48 | o : ~0ull, i};
        }
    });
    std::sort(ord.begin(), ord.end());
    // chunks of 256 objects in that order per task, each into its own buffer; stitched in input
    // order after
    std::vector<std::vector<u8>> part(nch);
    std::vector<u64> at(n);  // object i's bytes: part[chunk of its sorted position] at at[i]
    std::vector<u32> chunk_of(n);
    off[0] = 0;
    par_items(nch, nt, [&](size_t c, int tid) {
        if (!rds[tid]) rds[tid] = std::make_unique<Reader>(odb);
        Reader& rd = *rds[tid];
        std::vector<u8> buf;
        for (u64 s = c * CH; s < std::min(n, (c + 1) * CH); s++) {
            const u64 key = ord[s].first, i = ord[s].second;
            int type = 0;
            const int rc = key != ~0ull ? rd.read_packed(*odb->packs[key >> 48], key & ((1ull << 48) - 1), &type, buf)
                                        : rd.read(oids + 20 * i, &type, buf);
            status[i] = rc == RD_OK && type != OBJ_BLOB ? 2 : (u8)rc;
            if (status[i]) buf.clear();
            at[i] = part[c].size();
            chunk_of[i] = (u32)c;
            part[c].insert(part[c].end(), buf.begin(), buf.end());
            off[i + 1] = buf.size();  // lengths first, prefix-summed below
        }
    });
    for (u64 i = 0; i < n; i++) off[i + 1] += off[i];
    u8* p = (u8*)std::malloc(std::max<u64>(n ? off[n] : 0, 1));
    if (!p) { kd::set_error("kd_odb_read_batch: out of memory"); return KD_EINVAL; }
    par_items(nch, nt, [&](size_t c, int) {
        for (u64 i = c * CH; i < std::min(n, (c + 1) * CH); i++)
            if (off[i + 1] > off[i]) memcpy(p + off[i], part[chunk_of[i]].data() + at[i], off[i + 1] - off[i]);
    });
    *data = p;
    return KD_OK;
}

extern "C" int kd_walk(kd_odb* odb, const uint8_t* roots, int k, const char* subpath, int cmp0, int cmp1, int threads,
                       kd_leaves** out) {
    if (!odb || !roots || !out || k < 1 || k > KMAX) { kd::set_error("kd_walk: bad arguments"); return KD_EINVAL; }
    if ((cmp0 < 0) != (cmp1 < 0) || cmp0 >= k || cmp1 >= k || (cmp0 >= 0 && cmp0 == cmp1)) {
        kd::set_error("kd_walk: compare roots %d/%d of %d", cmp0, cmp1, k);
        return KD_EINVAL;
    }
    for (int r = 0; r < k && r < KMAX; r++) out[r] = nullptr;
    const int nt = default_threads(threads);
    Walk W;
    W.k = k;
    W.c0 = cmp0 < 0 ? -1 : cmp0;
    W.c1 = cmp1 < 0 ? -1 : cmp1;
    Reader rd0(odb);
    // ---- the walked tree of each root: peel commits, then follow `subpath` ----
    Item top;
    std::string msg;
    for (int r = 0; r < k && r < KMAX; r++) {
        int rc = peel_to_tree(rd0, roots + 20 * r, top.oid[r], msg);
        if (rc) { kd::set_error("kd_walk: %s", msg.c_str()); return rc; }
        top.has[r] = 1;
        top.mode[r] = 040000;
    }
    top.tree = true;
    const std::string sp = subpath ? subpath : "";
    size_t a = 0;
    std::vector<u8> buf;
    std::vector<TEnt> ents;
    while (a < sp.size()) {
        size_t b = sp.find('/', a);
        if (b == std::string::npos) b = sp.size();
        if (b > a) {
            const std::string comp = sp.substr(a, b - a);
            for (int r = 0; r < k && r < KMAX; r++) {
                if (!top.has[r]) continue;
                int type = 0;
                const int rc = rd0.read(top.oid[r], &type, buf);
                if (rc || type != OBJ_TREE || !parse_tree(buf, ents)) {
                    char hx[41];
                    hex40(top.oid[r], hx);
                    kd::set_error("kd_walk: cannot read tree %s", hx);
                    return rc == RD_MISSING ? KD_ENOTFOUND : KD_EINVAL;
                }
                top.has[r] = 0;
                for (const TEnt& e : ents)
                    if (e.tree() && e.nlen == comp.size() && !memcmp(e.name, comp.data(), e.nlen)) {
                        memcpy(top.oid[r], e.oid, 20);
                        top.has[r] = 1;
                        break;
                    }
            }
        }
        a = b + 1;
    }
    // ---- items: the top expanded breadth-first (in parallel) until there is work for every thread ----
    std::vector<Item> items;
    if (!W.pruned(top) && std::any_of(top.has, top.has + k, [](u8 h) { return h != 0; })) items.push_back(top);
    for (int level = 0; level < 4; level++) {
        size_t ntree = 0;
        for (auto& it : items) ntree += it.tree;
        if (ntree == 0 || ntree >= (size_t)nt * 16) break;
        std::vector<std::vector<Item>> kids(items.size());
        std::vector<std::unique_ptr<Reader>> rds(nt);
        par_items(items.size(), nt, [&](size_t i, int tid) {
            if (!items[i].tree) { kids[i].push_back(items[i]); return; }
            if (!rds[tid]) rds[tid] = std::make_unique<Reader>(odb);
            W.expand(*rds[tid], items[i], [&](const Item& c) { kids[i].push_back(c); });
        });
        if (W.err) break;
        std::vector<Item> next;
        for (auto& v : kids)
            for (auto& c : v) next.push_back(std::move(c));
        items.swap(next);
    }
    // ---- every item walked by some thread into its own outputs; then stitched in item order ----
    std::vector<WalkOut> outs;
    if (!W.err) {
        outs.resize(items.size() * k);
        std::vector<std::unique_ptr<Reader>> rds(nt);
        par_items(items.size(), nt, [&](size_t i, int tid) {
            WalkOut* o = &outs[i * k];
            if (!items[i].tree) { W.emit(items[i], o); return; }
            if (!rds[tid]) rds[tid] = std::make_unique<Reader>(odb);
            W.walk_item(*rds[tid], items[i], o);
        });
    }
    if (W.err) {
        kd::set_error("kd_walk: %s", W.emsg.c_str());
        return W.err.load();
    }
    for (int r = 0; r < k && r < KMAX; r++) {
        u64 n = 0, bytes = 0;
        for (size_t i = 0; i < items.size(); i++) {
            n += outs[i * k + r].end.size();
            bytes += outs[i * k + r].path.size();
        }
        // one block: header, path_off[n+1], mode[n], oid[20n], path bytes (kd_free)
        const size_t hsz = (sizeof(kd_leaves) + 15) & ~(size_t)15;
        const size_t total = hsz + 8 * (n + 1) + 4 * n + 20 * n + bytes + 16;
        u8* blk = (u8*)std::malloc(total);
        if (!blk) {
            for (int q = 0; q < r; q++) std::free(out[q]);
            kd::set_error("kd_walk: out of memory (%llu leaves)", (unsigned long long)n);
            return KD_EINVAL;
        }
        kd_leaves* L = (kd_leaves*)blk;
        L->n = n;
        L->path_off = (uint64_t*)(blk + hsz);
        L->mode = (uint32_t*)(L->path_off + n + 1);
        L->oid = (uint8_t*)(L->mode + n);
        L->path = L->oid + 20 * n;
        L->present = top.has[r];
        L->path_off[0] = 0;
        // per-item bases, then parallel copies
        std::vector<u64> lbase(items.size() + 1, 0), bbase(items.size() + 1, 0);
        for (size_t i = 0; i < items.size(); i++) {
            lbase[i + 1] = lbase[i] + outs[i * k + r].end.size();
            bbase[i + 1] = bbase[i] + outs[i * k + r].path.size();
        }
        par_items(items.size(), nt, [&](size_t i, int) {
            const WalkOut& o = outs[i * k + r];
            const u64 m = o.end.size();
            if (!m) return;
            memcpy(L->path + bbase[i], o.path.data(), o.path.size());
            memcpy(L->oid + 20 * lbase[i], o.oid.data(), 20 * m);
            memcpy(L->mode + lbase[i], o.mode.data(), 4 * m);
            for (u64 j = 0; j < m; j++) L->path_off[lbase[i] + j + 1] = bbase[i] + o.end[j];
        });
        out[r] = L;
    }
    return KD_OK;
}
