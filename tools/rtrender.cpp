// Headless driver (SURVEY 8(b) caller 1): .cli -> rt_* C ABI -> PNG (+ optional float RGB dump).
// The native counterpart of myRTFileReader's `write` command (myRTFileReader.java:86-93), which
// calls myScene.draw() and saves rndrdImg as PNG (myScene.java:1185-1196).
//
//   rtrender <scene_dir> <file.cli> [-w W] [-h H] [-spp N] [-seed S] [-device D] [-o out.png]
//            [-rgb out.f32] [-tex name=path.ppm]... [-time ITERS] [-nodir]
//
// Without -o the image goes where myScene.saveFile puts it (myScene.java:1185-1196): the
// `write` name (rt_scene_save_name) inside the folder "pics.<yyyy.MM.dd.hh.mm>" the scene
// creates (myScene.java:170, getDateTimeString :1329-1340; saveImgInDir defaults on :182),
// or in the current directory with -nodir. '/' separates the folder (the reference
// concatenates a Windows "\\").
//
// Textures are binary PPM (P6, 8-bit) files, one per texture name the .cli references
// (tools/textures_to_ppm.py converts the scene textures with the same decoder the tests use).
// Build: tools/build_rtrender.sh (links libdistraytracer.so and zlib).
#include <zlib.h>

#include <sys/stat.h>

#include <cstdio>
#include <ctime>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/distraytracer.h"

static bool read_ppm(const std::string& path, int& w, int& h, std::vector<uint8_t>& rgb) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  char magic[3] = {0};
  int maxv = 0;
  bool ok = std::fscanf(f, "%2s %d %d %d", magic, &w, &h, &maxv) == 4 && std::strcmp(magic, "P6") == 0 && maxv == 255;
  if (ok) {
    std::fgetc(f);  // single whitespace after the header
    rgb.resize((size_t)w * h * 3);
    ok = std::fread(rgb.data(), 1, rgb.size(), f) == rgb.size();
  }
  std::fclose(f);
  return ok;
}

static void be32(std::vector<uint8_t>& v, uint32_t x) {
  for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}
static void chunk(FILE* f, const char* type, const std::vector<uint8_t>& data) {
  std::vector<uint8_t> c;
  be32(c, (uint32_t)data.size());
  c.insert(c.end(), type, type + 4);
  c.insert(c.end(), data.begin(), data.end());
  uint32_t crc = crc32(0, c.data() + 4, (uInt)(c.size() - 4));
  be32(c, crc);
  std::fwrite(c.data(), 1, c.size(), f);
}
// PImage.save of rndrdImg: 8-bit RGB from the ARGB ints (myColor.getInt packing)
static bool write_png(const std::string& path, int w, int h, const int32_t* argb) {
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (w * 3 + 1));
  for (int y = 0; y < h; ++y) {
    raw.push_back(0);
    for (int x = 0; x < w; ++x) {
      uint32_t p = (uint32_t)argb[(size_t)y * w + x];
      raw.push_back((uint8_t)(p >> 16)); raw.push_back((uint8_t)(p >> 8)); raw.push_back((uint8_t)p);
    }
  }
  uLongf n = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(n);
  if (compress2(z.data(), &n, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
  z.resize(n);
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::fwrite(sig, 1, 8, f);
  std::vector<uint8_t> ihdr;
  be32(ihdr, (uint32_t)w);
  be32(ihdr, (uint32_t)h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit RGB
  chunk(f, "IHDR", ihdr);
  chunk(f, "IDAT", z);
  chunk(f, "IEND", {});
  return std::fclose(f) == 0;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <scene_dir> <file.cli> [-w W] [-h H] [-spp N] [-seed S] [-device D] "
                         "[-o out.png] [-rgb out.f32] [-tex name=path.ppm]... [-time ITERS] [-nodir]\n", argv[0]);
    return 2;
  }
  std::string dir = argv[1], cli = argv[2], out, rgbOut;
  bool inDir = true;
  int W = 300, H = 300, spp = 0, device = 0, timeIters = 0;  // DistRayTracer.java:15-16 default size
  uint64_t seed = 0x5EED0001ull;
  std::vector<std::string> texNames, texPaths;
  for (int i = 3; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "-w") W = std::atoi(next().c_str());
    else if (a == "-h") H = std::atoi(next().c_str());
    else if (a == "-spp") spp = std::atoi(next().c_str());
    else if (a == "-seed") seed = std::strtoull(next().c_str(), nullptr, 0);
    else if (a == "-device") device = std::atoi(next().c_str());
    else if (a == "-o") out = next();
    else if (a == "-rgb") rgbOut = next();
    else if (a == "-time") timeIters = std::atoi(next().c_str());
    else if (a == "-nodir") inDir = false;
    else if (a == "-tex") {
      std::string t = next();
      size_t eq = t.find('=');
      if (eq == std::string::npos) { std::fprintf(stderr, "-tex expects name=path.ppm\n"); return 2; }
      texNames.push_back(t.substr(0, eq));
      texPaths.push_back(t.substr(eq + 1));
    } else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
  }
  std::vector<std::vector<uint8_t>> texData(texNames.size());
  std::vector<rt_texture_desc> tex(texNames.size());
  std::vector<const char*> names(texNames.size());
  for (size_t t = 0; t < texNames.size(); ++t) {
    int w = 0, h = 0;
    if (!read_ppm(texPaths[t], w, h, texData[t])) { std::fprintf(stderr, "cannot read %s\n", texPaths[t].c_str()); return 1; }
    tex[t].w = w; tex[t].h = h; tex[t].rgb = texData[t].data();
    names[t] = texNames[t].c_str();
  }
  rt_scene* s = nullptr;
  int rc = rt_scene_load_cli(dir.c_str(), cli.c_str(), (int)tex.size(), names.data(), tex.data(), device, &s);
  if (rc) { std::fprintf(stderr, "rt_scene_load_cli: %d %s\n", rc, rt_last_error()); return 1; }
  if (out.empty()) {
    char name[4096];
    int n = rt_scene_save_name(s, name, (int)sizeof(name));
    if (n < 0 || n >= (int)sizeof(name)) { std::fprintf(stderr, "rt_scene_save_name: %s\n", rt_last_error()); return 1; }
    out = name;
    if (inDir) {
      std::time_t now = std::time(nullptr);
      std::tm tm = *std::localtime(&now);
      char folder[64];  // Calendar.HOUR: 12-hour clock, 0-11
      std::snprintf(folder, sizeof(folder), "pics.%d.%02d.%02d.%02d.%02d", tm.tm_year + 1900, tm.tm_mon + 1, tm.tm_mday,
                    tm.tm_hour % 12, tm.tm_min);
      mkdir(folder, 0755);
      out = std::string(folder) + "/" + out;
    }
  }
  rt_render_params p;
  std::memset(&p, 0, sizeof(p));
  p.width = W; p.height = H; p.spp = spp; p.row0 = 0; p.row1 = H; p.row_step = 1; p.seed = seed;
  std::vector<float> rgb((size_t)W * H * 3);
  std::vector<int32_t> argb((size_t)W * H);
  rc = rt_render(s, &p, rgb.data(), argb.data());
  if (rc) { std::fprintf(stderr, "rt_render: %d %s\n", rc, rt_last_error()); rt_scene_destroy(s); return 1; }
  if (timeIters > 0) {
    double ms = 0;
    rc = rt_time_render(s, &p, 1, timeIters, &ms);
    if (rc == 0) std::printf("render %dx%d: %.3f ms/frame (kernel, %d iters)\n", W, H, ms, timeIters);
  }
  rt_scene_destroy(s);
  if (!write_png(out, W, H, argb.data())) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); return 1; }
  if (!rgbOut.empty()) {
    FILE* f = std::fopen(rgbOut.c_str(), "wb");
    if (!f || std::fwrite(rgb.data(), sizeof(float), rgb.size(), f) != rgb.size()) return 1;
    std::fclose(f);
  }
  std::printf("wrote %s (%dx%d)\n", out.c_str(), W, H);
  return 0;
}
