// TF tensor-bundle checkpoint format (V2 Saver / tf.train.Checkpoint), written and read natively.
//
// Reference: the TF1 Saver the reference builds (reference trainer/task.py:143, task_supervisor.py:145
// with sharded=True) and the SavedModel variables/ directory (trainer/task.py:275-289) both produce
//   <prefix>.index                      SSTable: "" -> BundleHeaderProto, name -> BundleEntryProto
//   <prefix>.data-SSSSS-of-NNNNN        raw tensor bytes, one file per shard
// This file implements that layout from the format spec (LevelDB-style table: prefix-compressed
// blocks with restart points, 5-byte block trailer {type, masked crc32c}, metaindex + index blocks,
// 48-byte footer with magic 0xdb4775248b80fb57), hand-encoding the two small protobufs.
// Each entry carries the masked CRC32C of its bytes; reads verify it.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "runtime.h"

using namespace dtfrt;

namespace {

// ---------------------------------------------------------------- encoding helpers
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
void put_fixed32(std::string& s, uint32_t v) {
  char b[4];
  memcpy(b, &v, 4);
  s.append(b, 4);
}
void put_fixed64(std::string& s, uint64_t v) {
  char b[8];
  memcpy(b, &v, 8);
  s.append(b, 8);
}
bool get_varint(const char*& p, const char* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64 && p < end; shift += 7) {
    uint8_t b = (uint8_t)*p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}
uint32_t get_fixed32(const char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
// protobuf field helpers
void pb_varint(std::string& s, int field, uint64_t v) {
  put_varint(s, (uint64_t)field << 3 | 0);
  put_varint(s, v);
}
void pb_bytes(std::string& s, int field, const std::string& b) {
  put_varint(s, (uint64_t)field << 3 | 2);
  put_varint(s, b.size());
  s += b;
}
void pb_fixed32(std::string& s, int field, uint32_t v) {
  put_varint(s, (uint64_t)field << 3 | 5);
  put_fixed32(s, v);
}

struct Entry {
  int dtype = 0;
  std::vector<int64_t> dims;
  int shard = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;  // masked
};

std::string encode_entry(const Entry& e) {
  std::string s, shape;
  if (e.dtype) pb_varint(s, 1, (uint64_t)e.dtype);
  for (int64_t d : e.dims) {
    std::string dim;
    pb_varint(dim, 1, (uint64_t)d);
    pb_bytes(shape, 2, dim);
  }
  pb_bytes(s, 2, shape);
  if (e.shard) pb_varint(s, 3, (uint64_t)e.shard);
  if (e.offset) pb_varint(s, 4, (uint64_t)e.offset);
  if (e.size) pb_varint(s, 5, (uint64_t)e.size);
  pb_fixed32(s, 6, e.crc);
  return s;
}

std::string encode_header(int num_shards) {
  std::string s, ver;
  pb_varint(s, 1, (uint64_t)num_shards);
  // endianness LITTLE = 0 (default, omitted)
  pb_varint(ver, 1, 1);  // VersionDef.producer = 1
  pb_bytes(s, 3, ver);
  return s;
}

bool skip_field(const char*& p, const char* end, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(p, end, v);
    case 1: p += 8; return p <= end;
    case 2: if (!get_varint(p, end, v)) return false; p += v; return p <= end;
    case 5: p += 4; return p <= end;
  }
  return false;
}

bool decode_entry(const std::string& b, Entry& e) {
  const char* p = b.data();
  const char* end = p + b.size();
  while (p < end) {
    uint64_t key;
    if (!get_varint(p, end, key)) return false;
    int f = (int)(key >> 3), wt = (int)(key & 7);
    uint64_t v;
    if (f == 1 && wt == 0) { get_varint(p, end, v); e.dtype = (int)v; }
    else if (f == 2 && wt == 2) {
      get_varint(p, end, v);
      const char* se = p + v;
      while (p < se) {
        uint64_t k2;
        get_varint(p, se, k2);
        if ((k2 >> 3) == 2 && (k2 & 7) == 2) {
          uint64_t dl;
          get_varint(p, se, dl);
          const char* de = p + dl;
          int64_t size = 0;
          while (p < de) {
            uint64_t k3;
            get_varint(p, de, k3);
            if ((k3 >> 3) == 1 && (k3 & 7) == 0) { uint64_t sv; get_varint(p, de, sv); size = (int64_t)sv; }
            else if (!skip_field(p, de, (int)(k3 & 7))) return false;
          }
          e.dims.push_back(size);
        } else if (!skip_field(p, se, (int)(k2 & 7))) return false;
      }
    }
    else if (f == 3 && wt == 0) { get_varint(p, end, v); e.shard = (int)v; }
    else if (f == 4 && wt == 0) { get_varint(p, end, v); e.offset = (int64_t)v; }
    else if (f == 5 && wt == 0) { get_varint(p, end, v); e.size = (int64_t)v; }
    else if (f == 6 && wt == 5) { e.crc = get_fixed32(p); p += 4; }
    else if (!skip_field(p, end, wt)) return false;
  }
  return true;
}

// ---------------------------------------------------------------- SSTable writer
struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  std::string last_key;
  int counter = 0;
  int n = 0;
  static constexpr int kRestart = 16;
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < kRestart) {
      size_t m = std::min(last_key.size(), key.size());
      while (shared < m && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    put_varint(buf, shared);
    put_varint(buf, key.size() - shared);
    put_varint(buf, value.size());
    buf.append(key, shared, std::string::npos);
    buf += value;
    last_key = key;
    ++counter;
    ++n;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(out, r);
    put_fixed32(out, (uint32_t)restarts.size());
    return out;
  }
  void reset() {
    buf.clear();
    restarts.assign(1, 0);
    last_key.clear();
    counter = n = 0;
  }
};

struct TableWriter {
  FILE* f;
  uint64_t off = 0;
  BlockBuilder data, index;
  static constexpr size_t kBlockSize = 256 * 1024;
  explicit TableWriter(FILE* f_) : f(f_) {}
  std::string write_block(const std::string& contents) {
    std::string handle;
    put_varint(handle, off);
    put_varint(handle, contents.size());
    fwrite(contents.data(), 1, contents.size(), f);
    char trailer[5];
    trailer[0] = 0;  // no compression
    uint32_t crc = crc32c_extend(crc32c(contents.data(), contents.size()), trailer, 1);
    uint32_t m = crc_mask(crc);
    memcpy(trailer + 1, &m, 4);
    fwrite(trailer, 1, 5, f);
    off += contents.size() + 5;
    return handle;
  }
  void flush_data() {
    if (data.n == 0) return;
    std::string last = data.last_key;
    std::string h = write_block(data.finish());
    index.add(last, h);
    data.reset();
  }
  void add(const std::string& k, const std::string& v) {
    data.add(k, v);
    if (data.buf.size() >= kBlockSize) flush_data();
  }
  void finish() {
    flush_data();
    BlockBuilder meta;
    std::string mh = write_block(meta.finish());
    std::string ih = write_block(index.finish());
    std::string footer = mh + ih;
    footer.resize(40, '\0');
    put_fixed64(footer, 0xdb4775248b80fb57ull);
    fwrite(footer.data(), 1, footer.size(), f);
  }
};

// ---------------------------------------------------------------- SSTable reader
bool read_block(const std::string& file, uint64_t off, uint64_t size, std::string& out) {
  if (off + size + 5 > file.size()) return false;
  out.assign(file.data() + off, size);
  uint32_t want = crc_unmask(get_fixed32(file.data() + off + size + 1));
  uint32_t got = crc32c_extend(crc32c(file.data() + off, size), file.data() + off + size, 1);
  return want == got;
}

bool parse_block(const std::string& b, std::vector<std::pair<std::string, std::string>>& kv) {
  if (b.size() < 4) return false;
  uint32_t nr = get_fixed32(b.data() + b.size() - 4);
  size_t limit = b.size() - 4 - 4 * (size_t)nr;
  const char* p = b.data();
  const char* end = b.data() + limit;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint(p, end, shared) || !get_varint(p, end, nonshared) || !get_varint(p, end, vlen)) return false;
    if (p + nonshared + vlen > end || shared > key.size()) return false;
    key.resize(shared);
    key.append(p, nonshared);
    p += nonshared;
    kv.emplace_back(key, std::string(p, vlen));
    p += vlen;
  }
  return true;
}

bool read_file(const std::string& path, std::string& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  out.resize(n);
  size_t got = n ? fread(&out[0], 1, n, f) : 0;
  fclose(f);
  return (long)got == n;
}

std::string shard_name(const std::string& prefix, int i, int n) {
  char b[64];
  snprintf(b, sizeof b, ".data-%05d-of-%05d", i, n);
  return prefix + b;
}

// ---------------------------------------------------------------- objects
struct Writer {
  std::string prefix;
  int num_shards;
  std::vector<FILE*> files;
  std::vector<int64_t> offs;
  std::map<std::string, Entry> entries;
  bool failed = false;
};

struct Reader {
  std::string prefix;
  int num_shards = 1;
  std::map<std::string, Entry> entries;
  std::vector<std::string> names;
};

}  // namespace

DTF_RT void* dtfrt_bundle_writer_open(const char* prefix, int num_shards) {
  auto* w = new Writer;
  w->prefix = prefix;
  w->num_shards = num_shards < 1 ? 1 : num_shards;
  for (int i = 0; i < w->num_shards; ++i) {
    std::string p = shard_name(w->prefix, i, w->num_shards) + ".tmp";
    FILE* f = fopen(p.c_str(), "wb");
    if (!f) {
      set_error("cannot open %s", p.c_str());
      for (FILE* g : w->files) fclose(g);
      delete w;
      return nullptr;
    }
    w->files.push_back(f);
    w->offs.push_back(0);
  }
  return w;
}

// dtype: TF DataType enum (DT_FLOAT=1, DT_INT32=3, DT_INT64=9, DT_BFLOAT16=14, ...)
DTF_RT int dtfrt_bundle_add(void* h, const char* name, int dtype, int ndims, const int64_t* dims, const void* data,
                            int64_t nbytes, int shard) {
  auto* w = (Writer*)h;
  if (shard < 0 || shard >= w->num_shards) shard = 0;
  if (w->entries.count(name)) {
    set_error("duplicate tensor %s", name);
    return -1;
  }
  Entry e;
  e.dtype = dtype;
  e.dims.assign(dims, dims + ndims);
  e.shard = shard;
  e.offset = w->offs[shard];
  e.size = nbytes;
  e.crc = crc_mask(crc32c(data, (size_t)nbytes));
  if (nbytes && fwrite(data, 1, (size_t)nbytes, w->files[shard]) != (size_t)nbytes) {
    w->failed = true;
    set_error("short write for %s", name);
    return -2;
  }
  w->offs[shard] += nbytes;
  w->entries[name] = e;
  return 0;
}

// DT_STRING tensor: |varint64 len|... |masked crc32c of the length bytes| |bytes|...
DTF_RT int dtfrt_bundle_add_strings(void* h, const char* name, int ndims, const int64_t* dims, int n,
                                    const char* const* strs, const int64_t* lens, int shard) {
  std::string lenbuf, body;
  for (int i = 0; i < n; ++i) {
    put_varint(lenbuf, (uint64_t)lens[i]);
    body.append(strs[i], (size_t)lens[i]);
  }
  std::string all = lenbuf;
  put_fixed32(all, crc_mask(crc32c(lenbuf.data(), lenbuf.size())));
  all += body;
  return dtfrt_bundle_add(h, name, 7, ndims, dims, all.data(), (int64_t)all.size(), shard);
}

DTF_RT int dtfrt_bundle_finish(void* h) {
  auto* w = (Writer*)h;
  int rc = w->failed ? -1 : 0;
  for (FILE* f : w->files) {
    if (fclose(f) != 0) rc = -1;
  }
  std::string idx_tmp = w->prefix + ".index.tmp";
  FILE* f = fopen(idx_tmp.c_str(), "wb");
  if (!f) {
    set_error("cannot open %s", idx_tmp.c_str());
    delete w;
    return -1;
  }
  TableWriter tw(f);
  tw.add("", encode_header(w->num_shards));
  for (auto& kv : w->entries) tw.add(kv.first, encode_entry(kv.second));
  tw.finish();
  if (fclose(f) != 0) rc = -1;
  if (rc == 0) {  // publish atomically: data shards first, index last
    for (int i = 0; i < w->num_shards; ++i) {
      std::string p = shard_name(w->prefix, i, w->num_shards);
      rename((p + ".tmp").c_str(), p.c_str());
    }
    rename(idx_tmp.c_str(), (w->prefix + ".index").c_str());
  }
  delete w;
  return rc;
}

DTF_RT void* dtfrt_bundle_reader_open(const char* prefix) {
  std::string file;
  std::string path = std::string(prefix) + ".index";
  if (!read_file(path, file) || file.size() < 48) {
    set_error("cannot read %s", path.c_str());
    return nullptr;
  }
  const char* foot = file.data() + file.size() - 48;
  uint64_t magic;
  memcpy(&magic, foot + 40, 8);
  if (magic != 0xdb4775248b80fb57ull) {
    set_error("%s: bad table magic", path.c_str());
    return nullptr;
  }
  const char* p = foot;
  uint64_t mo, ms, io, is;
  get_varint(p, foot + 40, mo);
  get_varint(p, foot + 40, ms);
  get_varint(p, foot + 40, io);
  get_varint(p, foot + 40, is);
  std::string ib;
  if (!read_block(file, io, is, ib)) {
    set_error("%s: index block checksum mismatch", path.c_str());
    return nullptr;
  }
  std::vector<std::pair<std::string, std::string>> index_kv, kv;
  if (!parse_block(ib, index_kv)) {
    set_error("%s: corrupt index block", path.c_str());
    return nullptr;
  }
  for (auto& e : index_kv) {
    const char* hp = e.second.data();
    uint64_t bo, bs;
    get_varint(hp, hp + e.second.size(), bo);
    get_varint(hp, hp + e.second.size(), bs);
    std::string db;
    if (!read_block(file, bo, bs, db) || !parse_block(db, kv)) {
      set_error("%s: corrupt data block", path.c_str());
      return nullptr;
    }
  }
  auto* r = new Reader;
  r->prefix = prefix;
  for (auto& e : kv) {
    if (e.first.empty()) {  // header
      const char* q = e.second.data();
      const char* qe = q + e.second.size();
      while (q < qe) {
        uint64_t key;
        get_varint(q, qe, key);
        if ((key >> 3) == 1 && (key & 7) == 0) { uint64_t v; get_varint(q, qe, v); r->num_shards = (int)v; }
        else skip_field(q, qe, (int)(key & 7));
      }
      continue;
    }
    Entry en;
    if (!decode_entry(e.second, en)) {
      set_error("%s: bad entry for %s", path.c_str(), e.first.c_str());
      delete r;
      return nullptr;
    }
    r->entries[e.first] = en;
    r->names.push_back(e.first);
  }
  return r;
}

DTF_RT int dtfrt_bundle_num_tensors(void* h) { return (int)((Reader*)h)->names.size(); }
DTF_RT const char* dtfrt_bundle_name(void* h, int i) { return ((Reader*)h)->names[i].c_str(); }

DTF_RT int dtfrt_bundle_info(void* h, const char* name, int* dtype, int* ndims, int64_t* dims, int64_t* nbytes) {
  auto* r = (Reader*)h;
  auto it = r->entries.find(name);
  if (it == r->entries.end()) {
    set_error("tensor %s not found in %s", name, r->prefix.c_str());
    return -1;
  }
  const Entry& e = it->second;
  *dtype = e.dtype;
  *ndims = (int)e.dims.size();
  for (size_t i = 0; i < e.dims.size() && i < 16; ++i) dims[i] = e.dims[i];
  *nbytes = e.size;
  return 0;
}

DTF_RT int dtfrt_bundle_read(void* h, const char* name, void* dst, int64_t nbytes) {
  auto* r = (Reader*)h;
  auto it = r->entries.find(name);
  if (it == r->entries.end()) {
    set_error("tensor %s not found", name);
    return -1;
  }
  const Entry& e = it->second;
  if (nbytes < e.size) {
    set_error("buffer too small for %s", name);
    return -2;
  }
  std::string path = shard_name(r->prefix, e.shard, r->num_shards);
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    set_error("cannot open %s", path.c_str());
    return -3;
  }
  fseek(f, (long)e.offset, SEEK_SET);
  size_t got = e.size ? fread(dst, 1, (size_t)e.size, f) : 0;
  fclose(f);
  if ((int64_t)got != e.size) {
    set_error("short read for %s", name);
    return -4;
  }
  if (crc_mask(crc32c(dst, (size_t)e.size)) != e.crc) {
    set_error("checksum mismatch for %s", name);
    return -5;
  }
  return 0;
}

DTF_RT void dtfrt_bundle_reader_close(void* h) { delete (Reader*)h; }
