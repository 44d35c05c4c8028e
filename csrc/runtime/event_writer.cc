// TFRecord framing + TensorBoard event files (the reference's tf.summary.FileWriter,
// reference trainer/task.py:80,95,98: graph event + `loss` scalars at global_step).
//
// Record: uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)
// Event proto (hand-encoded): 1 wall_time double, 2 step int64, 3 file_version string,
// 4 graph_def bytes, 5 summary {1 value {1 tag, 2 simple_value float}}.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "runtime.h"

using namespace dtfrt;

namespace {

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
void put_tag(std::string& s, int f, int wt) { put_varint(s, (uint64_t)f << 3 | wt); }

struct RecWriter {
  FILE* f = nullptr;
  std::mutex mu;
};

int write_record(RecWriter* w, const void* data, uint64_t n) {
  std::lock_guard<std::mutex> g(w->mu);
  char hdr[12];
  memcpy(hdr, &n, 8);
  uint32_t c = crc_mask(crc32c(hdr, 8));
  memcpy(hdr + 8, &c, 4);
  uint32_t dc = crc_mask(crc32c(data, n));
  if (fwrite(hdr, 1, 12, w->f) != 12) return -1;
  if (n && fwrite(data, 1, n, w->f) != n) return -1;
  if (fwrite(&dc, 1, 4, w->f) != 4) return -1;
  return 0;
}

std::string event_header(double wall, int64_t step) {
  std::string e;
  put_tag(e, 1, 1);
  e.append((const char*)&wall, 8);
  if (step) {
    put_tag(e, 2, 0);
    put_varint(e, (uint64_t)step);
  }
  return e;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

struct RecReader {
  FILE* f = nullptr;
  std::string buf;
};

}  // namespace

DTF_RT void* dtfrt_tfrecord_writer_open(const char* path, int append) {
  FILE* f = fopen(path, append ? "ab" : "wb");
  if (!f) {
    set_error("cannot open %s", path);
    return nullptr;
  }
  auto* w = new RecWriter;
  w->f = f;
  return w;
}

DTF_RT int dtfrt_tfrecord_write(void* h, const void* data, uint64_t n) { return write_record((RecWriter*)h, data, n); }

DTF_RT int dtfrt_tfrecord_flush(void* h) {
  auto* w = (RecWriter*)h;
  std::lock_guard<std::mutex> g(w->mu);
  return fflush(w->f);
}

DTF_RT void dtfrt_tfrecord_writer_close(void* h) {
  auto* w = (RecWriter*)h;
  if (w->f) fclose(w->f);
  delete w;
}

// Event file = TFRecord file whose first record is Event{file_version: "brain.Event:2"}.
DTF_RT void* dtfrt_events_open(const char* path) {
  auto* w = (RecWriter*)dtfrt_tfrecord_writer_open(path, 0);
  if (!w) return nullptr;
  std::string e = event_header(now_s(), 0);
  std::string v = "brain.Event:2";
  put_tag(e, 3, 2);
  put_varint(e, v.size());
  e += v;
  write_record(w, e.data(), e.size());
  fflush(w->f);
  return w;
}

DTF_RT int dtfrt_events_scalar(void* h, const char* tag, float value, int64_t step, double wall) {
  std::string val, summ, e = event_header(wall > 0 ? wall : now_s(), step);
  size_t tl = strlen(tag);
  put_tag(val, 1, 2);
  put_varint(val, tl);
  val.append(tag, tl);
  put_tag(val, 2, 5);
  val.append((const char*)&value, 4);
  put_tag(summ, 1, 2);
  put_varint(summ, val.size());
  summ += val;
  put_tag(e, 5, 2);
  put_varint(e, summ.size());
  e += summ;
  return write_record((RecWriter*)h, e.data(), e.size());
}

// An Event carrying a serialized Summary (histograms, text, ...) built by the caller.
DTF_RT int dtfrt_events_summary(void* h, const void* summary, uint64_t n, int64_t step, double wall) {
  std::string e = event_header(wall > 0 ? wall : now_s(), step);
  put_tag(e, 5, 2);
  put_varint(e, n);
  e.append((const char*)summary, n);
  return write_record((RecWriter*)h, e.data(), e.size());
}

// Event.graph_def (field 4): a serialized graph description.
DTF_RT int dtfrt_events_graph(void* h, const void* graph, uint64_t n, double wall) {
  std::string e = event_header(wall > 0 ? wall : now_s(), 0);
  put_tag(e, 4, 2);
  put_varint(e, n);
  e.append((const char*)graph, n);
  return write_record((RecWriter*)h, e.data(), e.size());
}

DTF_RT void* dtfrt_tfrecord_reader_open(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    set_error("cannot open %s", path);
    return nullptr;
  }
  auto* r = new RecReader;
  r->f = f;
  return r;
}

// Returns 1 and sets *data/*n for the next record, 0 at EOF, <0 on corruption.
DTF_RT int dtfrt_tfrecord_next(void* h, const char** data, uint64_t* n) {
  auto* r = (RecReader*)h;
  char hdr[12];
  size_t got = fread(hdr, 1, 12, r->f);
  if (got == 0) return 0;
  if (got != 12) return -1;
  uint64_t len;
  memcpy(&len, hdr, 8);
  uint32_t lc;
  memcpy(&lc, hdr + 8, 4);
  if (crc_mask(crc32c(hdr, 8)) != lc) {
    set_error("tfrecord: length checksum mismatch");
    return -2;
  }
  r->buf.resize(len);
  if (len && fread(&r->buf[0], 1, len, r->f) != len) return -3;
  uint32_t dc;
  if (fread(&dc, 1, 4, r->f) != 4) return -3;
  if (crc_mask(crc32c(r->buf.data(), len)) != dc) {
    set_error("tfrecord: data checksum mismatch");
    return -4;
  }
  *data = r->buf.data();
  *n = len;
  return 1;
}

DTF_RT void dtfrt_tfrecord_reader_close(void* h) {
  auto* r = (RecReader*)h;
  fclose(r->f);
  delete r;
}
