// rv_container.hip -- the stream containers either side of the hot path
// (SURVEY.md §8f4): the y4m input the encoder reads and the IVF file it
// writes.  Host code only (no kernels); part of the library so a caller
// that drives the replay from a file needs nothing else.
//
// y4m: rav1e reads its input through the `y4m` crate (Decoder::new /
// read_frame, src/bin/decoder/y4m.rs:8-62); the crate is a third-party
// dependency absent from /root/reference, so the format is restated from its
// published definition: a stream header "YUV4MPEG2" followed by
// space-separated parameters (W width, H height, F num:den, I interlacing,
// A aspect, C colorspace, X comment) and '\n'; every frame "FRAME", optional
// parameters, '\n', then the planar samples Y, U, V (16-bit samples little
// endian above 8 bits).  Colorspaces map to rav1e's ChromaSampling as
// map_y4m_color_space does (src/bin/decoder/y4m.rs:78-93); a missing C is
// 4:2:0 8-bit.
//
// IVF: write_ivf_header / write_ivf_frame (ivf/src/lib.rs:6-30): "DKIF",
// version 0, header size 32, "AV01", width, height, framerate num, den, two
// zero words; each frame its length (u32), pts (u64), then its bytes; every
// field little endian.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "rv_device.h"

struct rv_y4m {
  FILE *f = nullptr;
  rv_y4m_info info;
  size_t frame_bytes = 0;
};

struct rv_ivf {
  FILE *f = nullptr;
  long frames = 0;
};

namespace {

// the header line's parameters (everything after "YUV4MPEG2")
int y4m_parse(const std::string &line, rv_y4m_info *o) {
  memset(o, 0, sizeof(*o));
  o->bit_depth = 8;
  o->xdec = o->ydec = 1;
  o->fps_num = 25;  // the crate's default when F is absent is irrelevant to the replay
  o->fps_den = 1;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && line[i] == ' ') i++;
    size_t j = i;
    while (j < line.size() && line[j] != ' ') j++;
    if (j > i) {
      const std::string tok = line.substr(i, j - i);
      const char k = tok[0];
      const std::string v = tok.substr(1);
      if (k == 'W') {
        o->width = atoi(v.c_str());
      } else if (k == 'H') {
        o->height = atoi(v.c_str());
      } else if (k == 'F') {
        const size_t c = v.find(':');
        if (c == std::string::npos) return rv_set_error(RV_EINVAL, "y4m: F needs num:den");
        o->fps_num = atoi(v.substr(0, c).c_str());
        o->fps_den = atoi(v.substr(c + 1).c_str());
      } else if (k == 'C') {
        // map_y4m_color_space: 420jpeg / 420paldv / 420mpeg2 / 420 are 4:2:0
        struct Cs {
          const char *name;
          int xdec, ydec, bd;
        };
        static const Cs kCs[] = {{"420jpeg", 1, 1, 8}, {"420paldv", 1, 1, 8}, {"420mpeg2", 1, 1, 8},
                                 {"420", 1, 1, 8},     {"420p10", 1, 1, 10},  {"420p12", 1, 1, 12},
                                 {"422", 1, 0, 8},     {"422p10", 1, 0, 10},  {"422p12", 1, 0, 12},
                                 {"444", 0, 0, 8},     {"444p10", 0, 0, 10},  {"444p12", 0, 0, 12}};
        bool found = false;
        for (const Cs &c : kCs)
          if (v == c.name) {
            o->xdec = c.xdec;
            o->ydec = c.ydec;
            o->bit_depth = c.bd;
            found = true;
          }
        if (!found) return rv_set_error(RV_EINVAL, "y4m: colorspace not supported (mono / unknown)");
      }  // I, A, X: not used by the encoder's input path
    }
    i = j;
  }
  if (o->width <= 0 || o->height <= 0 || o->fps_num <= 0 || o->fps_den <= 0)
    return rv_set_error(RV_EINVAL, "y4m: bad W / H / F");
  return RV_OK;
}

bool read_line(FILE *f, std::string *out, size_t cap) {
  out->clear();
  int c;
  while ((c = fgetc(f)) != EOF) {
    if (c == '\n') return true;
    if (out->size() >= cap) return false;
    out->push_back((char)c);
  }
  return false;
}

bool put_le(FILE *f, uint64_t v, int bytes) {
  uint8_t b[8];
  for (int i = 0; i < bytes; i++) b[i] = (uint8_t)(v >> (8 * i));
  return fwrite(b, 1, (size_t)bytes, f) == (size_t)bytes;
}

}  // namespace

extern "C" {

int rv_y4m_parse_header(const char *line, rv_y4m_info *out) {
  if (!line || !out) return rv_set_error(RV_EINVAL, "rv_y4m_parse_header: null");
  const std::string s(line);
  if (s.compare(0, 9, "YUV4MPEG2") != 0) return rv_set_error(RV_EINVAL, "y4m: not YUV4MPEG2");
  return y4m_parse(s.substr(9), out);
}

rv_y4m *rv_y4m_open(const char *path) {
  if (!path) {
    rv_set_error(RV_EINVAL, "rv_y4m_open: null path");
    return nullptr;
  }
  FILE *f = fopen(path, "rb");
  if (!f) {
    rv_set_error(RV_EINVAL, "rv_y4m_open: cannot open the file");
    return nullptr;
  }
  std::string line;
  rv_y4m_info info;
  if (!read_line(f, &line, 4096) || rv_y4m_parse_header(line.c_str(), &info) != RV_OK) {
    fclose(f);
    if (line.empty()) rv_set_error(RV_EINVAL, "y4m: no stream header");
    return nullptr;
  }
  rv_y4m *y = new rv_y4m();
  y->f = f;
  y->info = info;
  const size_t b = info.bit_depth > 8 ? 2 : 1;
  const size_t cw = (size_t)((info.width + info.xdec) >> info.xdec);
  const size_t ch = (size_t)((info.height + info.ydec) >> info.ydec);
  y->frame_bytes = b * ((size_t)info.width * info.height + 2 * cw * ch);
  return y;
}

int rv_y4m_get_info(const rv_y4m *y, rv_y4m_info *out) {
  if (!y || !out) return rv_set_error(RV_EINVAL, "rv_y4m_get_info: null");
  *out = y->info;
  return RV_OK;
}

size_t rv_y4m_frame_bytes(const rv_y4m *y) { return y ? y->frame_bytes : 0; }

int rv_y4m_read_frame(rv_y4m *y, void *host_yuv) {
  if (!y || !host_yuv) return rv_set_error(RV_EINVAL, "rv_y4m_read_frame: null");
  std::string line;
  if (!read_line(y->f, &line, 4096)) {
    if (line.empty() && feof(y->f)) return 1;  // the end of the stream
    return rv_set_error(RV_EINVAL, "y4m: truncated frame header");
  }
  if (line.compare(0, 5, "FRAME") != 0) return rv_set_error(RV_EINVAL, "y4m: expected FRAME");
  if (fread(host_yuv, 1, y->frame_bytes, y->f) != y->frame_bytes)
    return rv_set_error(RV_EINVAL, "y4m: truncated frame");
  return RV_OK;
}

void rv_y4m_close(rv_y4m *y) {
  if (!y) return;
  if (y->f) fclose(y->f);
  delete y;
}

rv_ivf *rv_ivf_create(const char *path, int width, int height, int fps_num, int fps_den) {
  if (!path || width <= 0 || width > 65535 || height <= 0 || height > 65535 || fps_num <= 0 ||
      fps_den <= 0) {
    rv_set_error(RV_EINVAL, "rv_ivf_create: bad arguments");
    return nullptr;
  }
  FILE *f = fopen(path, "wb");
  if (!f) {
    rv_set_error(RV_EINVAL, "rv_ivf_create: cannot create the file");
    return nullptr;
  }
  const bool ok = fwrite("DKIF", 1, 4, f) == 4 && put_le(f, 0, 2) && put_le(f, 32, 2) &&
                  fwrite("AV01", 1, 4, f) == 4 && put_le(f, (uint64_t)width, 2) &&
                  put_le(f, (uint64_t)height, 2) && put_le(f, (uint64_t)fps_num, 4) &&
                  put_le(f, (uint64_t)fps_den, 4) && put_le(f, 0, 4) && put_le(f, 0, 4);
  if (!ok) {
    fclose(f);
    rv_set_error(RV_EINVAL, "rv_ivf_create: write failed");
    return nullptr;
  }
  rv_ivf *v = new rv_ivf();
  v->f = f;
  return v;
}

int rv_ivf_write_frame(rv_ivf *v, uint64_t pts, const uint8_t *data, size_t len) {
  if (!v || (!data && len) || len > 0xffffffffu) return rv_set_error(RV_EINVAL, "rv_ivf_write_frame: bad arguments");
  if (!put_le(v->f, (uint64_t)len, 4) || !put_le(v->f, pts, 8) ||
      (len && fwrite(data, 1, len, v->f) != len))
    return rv_set_error(RV_EINVAL, "rv_ivf_write_frame: write failed");
  v->frames++;
  return RV_OK;
}

int rv_ivf_close(rv_ivf *v) {
  if (!v) return RV_OK;
  const int rc = fclose(v->f) == 0 ? RV_OK : rv_set_error(RV_EINVAL, "rv_ivf_close: close failed");
  delete v;
  return rc;
}

}  // extern "C"
