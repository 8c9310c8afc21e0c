// Native mirror of the reference's `.cli` reader, myRTFileReader.readRTFile
// (src/rayTracerDistAccelShdPhtnMap/myRTFileReader.java:15-349), and of the
// builder state it drives in myScene (myScene.java:144-145 material state,
// :305-324 accel lists, :413-444 lights, :447-521 prims, :1235-1323 matrix
// stack). It emits the flattened rt_scene_desc that a JNI myScene subclass
// would hand over, then calls rt_scene_create().
//
// Unknown commands are reported on stderr and skipped, as readRTFile's default case does
// (myRTFileReader.java:343-345); malformed arguments of known commands fail with RT_E_PARSE.
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/distraytracer.h"
#include "host_math.h"
#include "rt_internal.h"

namespace rt {
using namespace hm;

namespace {

struct Clr {
  double r = 0, g = 0, b = 0;
};
static Clr clr(double r, double g, double b) { return Clr{jmin(1, r), jmin(1, g), jmin(1, b)}; }  // myColor clamp

// DistRayTracer.getClr (DistRayTracer.java:467-530): named colours of `noise_color`
// (clr_rnd draws from Processing's unseeded random: rejected)
static bool named_color(std::string n, Clr& c) {
  for (auto& ch : n) ch = (char)std::tolower(ch);
  static const std::map<std::string, Clr> tab = {
      {"clr_gray", {0.47, 0.47, 0.47}}, {"clr_white", {1.0, 1.0, 1.0}}, {"clr_yellow", {1.0, 1.0, 0}},
      {"clr_cyan", {0, 1.0, 1.0}}, {"clr_magenta", {1.0, 0, 1.0}}, {"clr_red", {1.0, 0, 0}}, {"clr_blue", {0, 0, 1.0}},
      {"clr_purple", {0.6, 0.2, 1.0}}, {"clr_green", {0, 1.0, 0}}, {"clr_ltwood1", {0.94, 0.47, 0.12}},
      {"clr_ltwood2", {0.94, 0.8, 0.4}}, {"clr_dkwood1", {0.2, 0.08, 0.08}}, {"clr_dkwood2", {0.3, 0.20, 0.16}},
      {"clr_mortar1", {0.2, 0.2, 0.2}}, {"clr_mortar2", {0.7, 0.7, 0.7}}, {"clr_brick1_1", {0.6, 0.18, 0.22}},
      {"clr_brick1_2", {0.8, 0.26, 0.33}}, {"clr_brick2_1", {0.6, 0.32, 0.16}}, {"clr_brick2_2", {0.8, 0.45, 0.25}},
      {"clr_brick3_1", {0.3, 0.01, 0.07}}, {"clr_brick3_2", {0.6, 0.02, 0.13}}, {"clr_brick4_1", {0.4, 0.1, 0.17}},
      {"clr_brick4_2", {0.6, 0.3, 0.13}}, {"clr_darkgray", {0.31, 0.31, 0.31}}, {"clr_darkred", {0.47, 0, 0}},
      {"clr_darkblue", {0, 0, 0.47}}, {"clr_darkpurple", {0.4, 0.2, 0.6}}, {"clr_darkgreen", {0, 0.47, 0}},
      {"clr_darkyellow", {0.47, 0.47, 0}}, {"clr_darkmagenta", {0.47, 0, 0.47}}, {"clr_darkcyan", {0, 0.47, 0.47}},
      {"clr_lightgray", {0.78, 0.78, 0.78}}, {"clr_lightred", {1.0, .43, .43}}, {"clr_lightblue", {0.43, 0.43, 1.0}},
      {"clr_lightgreen", {0.43, 1.0, 0.43}}, {"clr_lightyellow", {1.0, 1.0, .43}}, {"clr_lightmagenta", {1.0, .43, 1.0}},
      {"clr_lightcyan", {0.43, 1.0, 1.0}}, {"clr_black", {0, 0, 0}}, {"clr_nearblack", {0.05, 0.05, 0.05}},
      {"clr_faintgray", {0.43, 0.43, 0.43}}, {"clr_faintred", {0.43, 0, 0}}, {"clr_faintblue", {0, 0, 0.43}},
      {"clr_faintgreen", {0, 0.43, 0}}, {"clr_faintyellow", {0.43, 0.43, 0}}, {"clr_faintcyan", {0, 0.43, 0.43}},
      {"clr_faintmagenta", {0.43, 0, 0.43}}, {"clr_offwhite", {0.95, 0.98, 0.92}}};
  auto it = tab.find(n);
  if (it != tab.end()) { c = it->second; return true; }
  if (n == "clr_rnd") return false;
  c = clr(1.0, 1.0, 1.0);  // "Color not found ... so using white"
  return true;
}

struct CliLoader {
  std::string dir, saveName;
  int ignored = 0;  // unknown commands skipped (myRTFileReader.java:343-345)
  int refine = -1;  // `refine on|off` (myScene.setRefine, myRTFileReader.java:111); -1 = not given
  std::map<std::string, int> texIndex;
  std::vector<Mat> stack{Mat::ident()};
  // material state
  Clr cDiff, cAmb, cSpec, permClr, kReflClr;
  double phong = 0, kRefl = 0, kTrans = 0, rfrIdx = 0;
  bool simple = false, txTop = false;
  int txtrType = 0;
  int texTop = -1;
  double noiseScale = 1, turbMult = 1, colorScale = 10, colorMult = .2;
  int octaves = 8;
  D3 pdMult{10, 10, 10};
  bool rndColors = false, useFwdTrans = false, useCustClrs = false;
  std::vector<Clr> noiseColors{clr(.7, .7, .7), clr(.2, .2, .2)};
  int numPtsDist = 2, distFunc = 1, roiFunc = 1;
  double avgNumPerCell = 1.0, mortarThresh = 0.05;
  bool photonMap = false, caustic = false;
  // accumulated desc
  std::vector<rt_prim_desc> prims;
  std::vector<rt_material_desc> mats;
  std::vector<rt_light_desc> lights;
  std::vector<rt_accel_desc> accels;
  std::vector<int32_t> members, top;
  std::vector<rt_instance_desc> insts;
  std::map<std::string, int32_t> named;  // namedObjs (myScene.java:378-387): prim index or ~accel
  bool lastWasLight = false;             // allObjsToFind's last entry is a light
  bool inList = false;
  std::vector<int32_t> tmp;
  rt_scene_desc d{};
  int curRpp = 0;
  std::string err;

  void put_ctm(double* dst) { std::memcpy(dst, stack.back().m, sizeof(double) * 16); }
  void set_surface(Clr df, Clr am, Clr sp, double ph, double kr) {  // myScene.setSurface :817-828
    txtrType = 0;
    cDiff = df; cAmb = am; cSpec = sp; phong = ph;
    kRefl = kr; kReflClr = clr(kr, kr, kr);
    rfrIdx = 0; permClr = clr(0, 0, 0); kTrans = 0;
  }
  int material() {  // getCurShader (myScene.java:524-542): a fresh shader per object, dedup by value
    rt_material_desc m;
    std::memset(&m, 0, sizeof(m));
    m.simple = simple;
    m.texture = (txtrType >= 1 && txtrType <= 6) ? txtrType : RT_TEX_NONE;
    m.tex_top = (txtrType == 1 && txTop) ? texTop : -1;
    m.use_photon_map = photonMap;
    m.caustic_photons = caustic;
    m.diffuse[0] = cDiff.r; m.diffuse[1] = cDiff.g; m.diffuse[2] = cDiff.b;
    m.ambient[0] = cAmb.r; m.ambient[1] = cAmb.g; m.ambient[2] = cAmb.b;
    m.specular[0] = cSpec.r; m.specular[1] = cSpec.g; m.specular[2] = cSpec.b;
    m.phong_exp = phong;
    m.k_refl = kRefl;
    m.k_refl_clr[0] = kReflClr.r; m.k_refl_clr[1] = kReflClr.g; m.k_refl_clr[2] = kReflClr.b;
    m.k_trans = kTrans;
    m.perm = rfrIdx;
    m.perm_clr[0] = permClr.r; m.perm_clr[1] = permClr.g; m.perm_clr[2] = permClr.b;
    if (txtrType >= 2 && txtrType <= 6) {
      m.noise_scale = noiseScale; m.turb_mult = turbMult; m.color_scale = colorScale; m.color_mult = colorMult;
      m.period_mult[0] = pdMult.x; m.period_mult[1] = pdMult.y; m.period_mult[2] = pdMult.z;
      m.octaves = octaves; m.rnd_colors = rndColors; m.use_fwd_trans = useFwdTrans;
      std::vector<Clr> cl = noiseColors;
      while (cl.size() < 2) cl.push_back(clr(1, 1, 1));  // (Java would throw at render)
      m.num_colors = (int32_t)std::min<size_t>(cl.size(), RT_MAX_NOISE_COLORS);
      for (int i = 0; i < m.num_colors; ++i) { m.colors[i][0] = cl[i].r; m.colors[i][1] = cl[i].g; m.colors[i][2] = cl[i].b; }
      if (txtrType == RT_TEX_STONE) {
        m.dist_func = distFunc; m.roi_func = roiFunc; m.num_pts_dist = numPtsDist;
        m.avg_per_cell = avgNumPerCell; m.mortar_thresh = mortarThresh;
      }
    }
    for (size_t i = 0; i < mats.size(); ++i)
      if (std::memcmp(&mats[i], &m, sizeof(m)) == 0) return (int)i;
    mats.push_back(m);
    return (int)mats.size() - 1;
  }
  void add_prim(rt_prim_desc& p) {  // addObjectToScene (myScene.java:558-565)
    p.material = material();
    int idx = (int)prims.size();
    prims.push_back(p);
    if (inList) tmp.push_back(idx);
    else top.push_back(idx);
    lastWasLight = false;
  }
  // gtTranslate / gtScale / gtRotate (myScene.java:1256-1318)
  void translate(double x, double y, double z) {
    Mat T = Mat::ident();
    T.m[3] = x; T.m[7] = y; T.m[11] = z;
    stack.back() = mul(stack.back(), T);
  }
  void scale(double x, double y, double z) {
    Mat S = Mat::ident();
    S.m[0] = x; S.m[5] = y; S.m[10] = z;
    stack.back() = mul(stack.back(), S);
  }
  void rotate(double ang, double ax, double ay, double az) {
    double ar = (double)(ang * M_PI) / 180.0;
    D3 av = normalized(d3(ax, ay, az));
    D3 nv = (ax == 0) ? d3(1, 0, 0) : d3(0, 1, 0);
    D3 bv = normalized(cross(av, nv));
    D3 cv = normalized(cross(av, bv));
    Mat R1 = Mat::ident(), R2 = Mat::ident();
    R1.m[0] = av.x; R1.m[1] = av.y; R1.m[2] = av.z;
    R1.m[4] = bv.x; R1.m[5] = bv.y; R1.m[6] = bv.z;
    R1.m[8] = cv.x; R1.m[9] = cv.y; R1.m[10] = cv.z;
    R2.m[5] = jf::cos(ar); R2.m[6] = -jf::sin(ar); R2.m[9] = jf::sin(ar); R2.m[10] = jf::cos(ar);
    stack.back() = mul(stack.back(), mul(transpose(R1), mul(R2, R1)));
  }
  void push() { stack.push_back(stack.back()); }  // gtPushMatrix :1241-1246
  void pop() { if (stack.size() > 1) stack.pop_back(); }
  // addInstance (myScene.java:389-395) + myInstance ctor (mySceneObject.java:98-110)
  bool add_instance(const std::string& name, bool addShdr) {
    auto it = named.find(name);
    if (it == named.end()) { err = "unknown named object: " + name; return false; }
    rt_instance_desc in;
    std::memset(&in, 0, sizeof(in));
    in.base = it->second;
    Mat bg;
    std::memcpy(bg.m, in.base >= 0 ? prims[in.base].ctm : accels[~in.base].ctm, sizeof(bg.m));
    Mat g = mul(bg, stack.back());  // buildCTMara(scene, obj.CTMara[glbl]) = obj glbl x stack top
    std::memcpy(in.ctm, g.m, sizeof(in.ctm));
    D3 o = xform(stack.back(), d3(0, 0, 0), 1);
    in.origin[0] = o.x; in.origin[1] = o.y; in.origin[2] = o.z;
    in.material = addShdr ? material() : -1;  // useInstShader: getCurShader()
    int32_t ref = RT_INSTANCE_REF((int32_t)insts.size());
    insts.push_back(in);
    if (inList) tmp.push_back(ref);
    else top.push_back(ref);
    lastWasLight = false;
    return true;
  }
  // setSierpShdr (myScene.java:328-337), float arithmetic as in the reference
  void sierp_shader(int level, int maxLevel) {
    float bVal = 1.0f - std::min(1.0f, (1.5f * level / maxLevel)), rVal = 1.0f - bVal,
          tmpv = std::min((1.2f * (level - (maxLevel / 2))) / (1.0f * maxLevel), 1.0f), gVal = (tmpv * tmpv);
    txTop = false;
    set_surface(clr(std::min(1.0f, rVal + .5f), std::min(1.0f, gVal + .5f), std::min(1.0f, bVal + .5f)), clr(0, 0, 0),
                clr(0, 0, 0), 0, 0);
  }
  void sierp_shift(float newTrans) { rotate(120, 1, 0, 0); translate(0, newTrans, 0); rotate(-120, 1, 0, 0); }
  // buildSierpSubTri (myScene.java:339-369): one instance per call, then four scaled sub-tetrahedra
  bool sierp_sub(float dim, float scVal, const std::string& name, int level, int maxLevel, bool addShader) {
    if (level >= maxLevel) return true;
    float newDim = scVal * dim;
    push();
    translate(0, .1f * dim, 0);
    rotate(70, 0, 1, 0);
    if (addShader) sierp_shader(level, maxLevel);
    if (!add_instance(name, addShader)) return false;
    pop();
    const float sqrt66 = (float)std::sqrt(6.0f) / 6.0f;  // DistRayTracer.java:38
    float newTrans = sqrt66 * dim;
    for (int k = 0; k < 4; ++k) {  // up, front, left, right
      push();
      if (k == 0) translate(0, newTrans, 0);
      else if (k == 1) sierp_shift(newTrans);
      else if (k == 2) { rotate(120, 0, 1, 0); sierp_shift(newTrans); rotate(-120, 0, 1, 0); }
      else { rotate(-120, 0, 1, 0); sierp_shift(newTrans); rotate(120, 0, 1, 0); }
      scale(scVal, scVal, scVal);
      if (!sierp_sub(newDim, scVal, name, level + 1, maxLevel, addShader)) return false;
      pop();
    }
    return true;
  }
  void end_list(bool bvh) {  // endTmpObjList (myScene.java:305-324)
    inList = false;
    rt_accel_desc a;
    std::memset(&a, 0, sizeof(a));
    a.type = bvh ? 1 : 0;
    a.first = (int)members.size();
    a.count = (int)tmp.size();
    put_ctm(a.ctm);
    members.insert(members.end(), tmp.begin(), tmp.end());
    top.push_back(~(int32_t)accels.size());
    accels.push_back(a);
    tmp.clear();
    lastWasLight = false;
  }
  rt_prim_desc new_prim(int type) {
    rt_prim_desc p;
    std::memset(&p, 0, sizeof(p));
    p.type = type;
    put_ctm(p.ctm);
    return p;
  }
  void reset_dflt_txtr() {  // resetDfltTxtrVals (myScene.java:579-586)
    txtrType = 0; octaves = 4; rndColors = false; useCustClrs = false; useFwdTrans = false;
    noiseScale = 1.0; turbMult = 1.0; colorScale = 5.0; colorMult = .1;
    pdMult = d3(1.0, 1.0, 1.0);
    noiseColors = {clr(0.05, 0.05, 0.05), clr(1.0, 1.0, 1.0)};
    numPtsDist = 2; distFunc = 1; roiFunc = 1; avgNumPerCell = 1.0; mortarThresh = 0.05;
  }
  bool read_worley(const std::vector<std::string>& v) {  // readProcTxtrWorleyVals (myScene.java:675-708)
    try {
      size_t k = 1;
      noiseScale = num(v, k++);
      distFunc = std::stoi(v.at(k++));
      roiFunc = std::stoi(v.at(k++));
      numPtsDist = std::stoi(v.at(k++));
      avgNumPerCell = num(v, k++);
      mortarThresh = num(v, k++);
      useFwdTrans = (num(v, k++) == 1.0);
      if (v.size() >= k + 2) {
        colorScale = num(v, k); colorMult = num(v, k + 1); rndColors = true;
      } else {
        rndColors = false; colorScale = 25.0; colorMult = .1;
      }
      return false;
    } catch (...) {
      return true;
    }
  }
  static double num(const std::vector<std::string>& t, size_t i) {
    if (i >= t.size()) throw std::out_of_range("missing argument");
    return std::stod(t[i]);
  }
  bool read_perlin(const std::vector<std::string>& v) {  // readProcTxtrPerlinVals (myScene.java:642-672)
    try {
      if (v.size() < 11) return true;
      noiseScale = num(v, 1); octaves = std::stoi(v.at(2)); turbMult = num(v, 3);
      pdMult = d3(num(v, 4), num(v, 5), num(v, 6));
      D3 py = d3(num(v, 7), num(v, 8), num(v, 9));
      if (((py.x * py.x) + (py.y * py.y)) + (py.z * py.z) > 0) {
        py = d3(py.x * (TWO_PI_F - 1.0), py.y * (TWO_PI_F - 1.0), py.z * (TWO_PI_F - 1.0));
        py = d3(py.x + 1.0, py.y + 1.0, py.z + 1.0);
        pdMult = d3(pdMult.x * py.x, pdMult.y * py.y, pdMult.z * py.z);
      }
      useFwdTrans = (num(v, 10) == 1.0);
      if (v.size() >= 13) {
        colorScale = num(v, 11); colorMult = num(v, 12); rndColors = true;
      } else {
        rndColors = false; colorScale = 25.0; colorMult = .1;
      }
      return false;
    } catch (...) {
      return true;
    }
  }

  bool read(const std::string& fname, bool isMain) {
    std::ifstream f(dir + "/" + fname);
    if (!f) { err = "cannot open " + dir + "/" + fname; return false; }
    std::string line;
    rt_prim_desc poly;
    bool inPoly = false;
    int vc = 0;
    int lineNo = -1;
    while (std::getline(f, line)) {
      ++lineNo;
      std::vector<std::string> t;
      {  // PApplet.splitTokens(line, " ")
        std::string cur;
        for (char ch : line) {
          if (ch == ' ' || ch == '\t' || ch == '\r') { if (!cur.empty()) { t.push_back(cur); cur.clear(); } }
          else cur.push_back(ch);
        }
        if (!cur.empty()) t.push_back(cur);
      }
      if (t.empty() || t[0][0] == '#') continue;
      const std::string& c = t[0];
      try {
        if (c == "fov") {  // :51-58
          if (!isMain) continue;
          d.rays_per_pixel = (curRpp != 0) ? curRpp : 1;
          d.fov = num(t, 1);
          d.camera = RT_CAMERA_FOV;
        } else if (c == "fisheye" || c == "fishEye") {  // :66-74 (myFishEyeScene)
          if (!isMain) continue;
          d.rays_per_pixel = (curRpp != 0) ? curRpp : 1;
          d.camera = RT_CAMERA_FISHEYE;
          d.camera_param[0] = num(t, 1);
          d.camera_param[1] = 0;
        } else if (c == "ortho" || c == "orthographic") {  // :75-83 (myOrthoScene)
          if (!isMain) continue;
          d.rays_per_pixel = (curRpp != 0) ? curRpp : 1;
          d.camera = RT_CAMERA_ORTHO;
          d.camera_param[0] = num(t, 1);
          d.camera_param[1] = num(t, 2);
        } else if (c == "lens") {
          d.dof = 1; d.lens_radius = num(t, 1); d.lens_focal = num(t, 2);
        } else if (c == "write") {
          if (saveName.empty()) saveName = t.at(1);  // scene.saveName (:87)
          break;  // the reference renders here (:86-93)
        } else if (c == "read") {
          if (!read(t.at(1), false)) return false;
        } else if (c == "rays_per_pixel") {
          curRpp = std::stoi(t.at(1)); d.rays_per_pixel = curRpp;
        } else if (c == "antialias") {
          curRpp = std::stoi(t.at(1)) * std::stoi(t.at(2)); d.rays_per_pixel = curRpp;
        } else if (c == "background") {  // :129-148
          if (t.at(1) == "texture") {
            auto it = texIndex.find(t.at(2));
            if (it == texIndex.end()) { err = "texture not registered: " + t.at(2); return false; }
            d.bkg_texture = it->second;
            d.skydome[0] = num(t, 3); d.skydome[1] = num(t, 4); d.skydome[2] = num(t, 5); d.skydome[3] = num(t, 6);
          } else {
            Clr b = clr(num(t, 1), num(t, 2), num(t, 3));
            d.background[0] = b.r; d.background[1] = b.g; d.background[2] = b.b;
            txtrType = 0;
          }
        } else if (c == "point_light" || c == "spotlight" || c == "disk_light") {  // myScene.java:413-444
          if (inList) { err = "light inside accel list unsupported"; return false; }
          rt_light_desc L;
          std::memset(&L, 0, sizeof(L));
          put_ctm(L.ctm);
          L.pos[0] = num(t, 1); L.pos[1] = num(t, 2); L.pos[2] = num(t, 3);
          Clr col;
          if (c == "point_light") {
            L.type = RT_LIGHT_POINT;
            col = clr(num(t, 4), num(t, 5), num(t, 6));
          } else if (c == "spotlight") {
            L.type = RT_LIGHT_SPOT;
            L.dir[0] = num(t, 4); L.dir[1] = num(t, 5); L.dir[2] = num(t, 6);
            L.inner_deg = num(t, 7); L.outer_deg = num(t, 8);
            col = clr(num(t, 9), num(t, 10), num(t, 11));
          } else {
            L.type = RT_LIGHT_DISK;
            L.radius = num(t, 4);
            L.dir[0] = num(t, 5); L.dir[1] = num(t, 6); L.dir[2] = num(t, 7);
            col = clr(num(t, 8), num(t, 9), num(t, 10));
          }
          L.color[0] = col.r; L.color[1] = col.g; L.color[2] = col.b;
          lights.push_back(L);
          lastWasLight = true;
        } else if (c == "caustic_photons" || c == "diffuse_photons") {  // setPhotonHandling :919-931
          photonMap = true;
          caustic = (c.find("caustic") != std::string::npos);
          d.photon_mode = caustic ? 2 : 1;
          d.photon_count = std::stoi(t.at(1));
          d.photon_k = std::stoi(t.at(2));
          d.photon_max_dist = (double)std::stof(t.at(3));
        } else if (c == "final_gather") {
        } else if (c == "diffuse" || c == "reflective") {
          txTop = false;
          set_surface(clr(num(t, 1), num(t, 2), num(t, 3)), clr(num(t, 4), num(t, 5), num(t, 6)), clr(0, 0, 0), 0,
                      c == "reflective" ? num(t, 7) : 0);
        } else if (c == "shiny" || c == "surface") {  // setSurfaceShiny (myRTFileReader.java:358-378)
          Clr df = clr(num(t, 1), num(t, 2), num(t, 3)), am = clr(num(t, 4), num(t, 5), num(t, 6)),
              sp = clr(num(t, 7), num(t, 8), num(t, 9));
          double ph = num(t, 10), kr = num(t, 11), kt = 0, ri = 0;
          txTop = false;
          set_surface(df, am, sp, ph, kr);
          if (t.size() > 12) {
            kt = num(t, 12);
            kTrans = kt;
            if (t.size() > 13) {
              ri = num(t, 13);
              rfrIdx = ri; permClr = clr(ri, ri, ri);
              if (t.size() > 16) permClr = clr(num(t, 14), num(t, 15), num(t, 16));
            }
          }
          if (c == "shiny" && ((kt > 0) || (ri > 0))) simple = true;
        } else if (c == "perm") {
          rfrIdx = num(t, 1); permClr = clr(rfrIdx, rfrIdx, rfrIdx);
          if (t.size() > 4) permClr = clr(num(t, 2), num(t, 3), num(t, 4));
        } else if (c == "phong") { phong = num(t, 1);
        } else if (c == "krefl") { kRefl = num(t, 1); kReflClr = clr(kRefl, kRefl, kRefl);
        } else if (c == "ktrans") { kTrans = num(t, 1);
        } else if (c == "depth") {
        } else if (c == "begin_list") {
          inList = true; tmp.clear();
        } else if (c == "end_list" || c == "end_accel") {
          end_list(c == "end_accel");
        } else if (c == "named_object") {  // setObjectAsNamedObject (myScene.java:378-387)
          if (inList || top.empty() || lastWasLight) { err = "named_object: only a scene object (not a light) can be named"; return false; }
          int32_t v = top.back();
          if (v >= 0 && (v & RT_REF_INSTANCE)) { err = "named_object of an instance is unsupported"; return false; }
          top.pop_back();
          named[t.at(1)] = v;
        } else if (c == "instance") {  // myRTFileReader.java:250-256: any 3rd token selects the current shader
          if (!add_instance(t.at(1), t.size() > 2)) return false;
        } else if (c == "sierpinski") {  // myRTFileReader.java:234-241, buildSierpinski (myScene.java:371-377)
          std::string objName = t.at(1);
          float sc = .5f;
          int depth = 5;
          bool useShdr = false;  // useShdr != "No": true iff a 5th token was parsed
          try {
            depth = std::stoi(t.at(2));
            sc = std::stof(t.at(3));
            useShdr = t.size() > 4;
          } catch (...) {
          }
          if (inList) { err = "sierpinski inside begin_list is unsupported"; return false; }
          inList = true; tmp.clear();  // startTmpObjList
          if (!sierp_sub(8, sc, objName, 0, depth, useShdr)) return false;
          end_list(true);
        } else if (c == "texture" || c == "image_texture") {  // :257-273
          std::string lo = t.at(1);
          for (auto& ch : lo) ch = (char)std::tolower(ch);
          if (lo == "top" || lo != "bottom") {
            std::string name = (lo == "top") ? t.at(2) : t.at(1);
            auto it = texIndex.find(name);
            if (it == texIndex.end()) { err = "texture not registered: " + name; return false; }
            texTop = it->second;
            txTop = true;
          }
          txtrType = 1;
        } else if (c == "noise") {
          reset_dflt_txtr(); txtrType = 2; noiseScale = num(t, 1);
        } else if (c == "marble") {  // setTexture (myScene.java:743-755)
          reset_dflt_txtr();
          txtrType = 4;
          bool dflt = read_perlin(t);
          if (!useCustClrs) noiseColors = {clr(0.05, 0.05, 0.05), clr(0.95, 0.98, 0.92)};
          if (dflt) {
            octaves = 16; rndColors = true; useFwdTrans = false;
            noiseScale = 1.0; turbMult = 15.0; colorScale = 24.0; colorMult = .1;
            pdMult = d3(TWO_PI_F * 0.1, TWO_PI_F * 31.4, TWO_PI_F * 4.1);
          }
        } else if (c == "wood" || c == "wood2") {  // setTexture (myScene.java:717-742)
          reset_dflt_txtr();
          const bool w2 = c == "wood2";
          txtrType = w2 ? RT_TEX_WOOD2 : RT_TEX_WOOD;
          bool dflt = read_perlin(t);
          if (!useCustClrs) {
            noiseColors = w2 ? std::vector<Clr>{clr(0.3, 0.20, 0.16), clr(0.94, 0.8, 0.4)}      // clr_dkwood2, clr_ltwood2
                             : std::vector<Clr>{clr(0.2, 0.08, 0.08), clr(0.94, 0.47, 0.12)};  // clr_dkwood1, clr_ltwood1
          }
          if (dflt) {
            octaves = w2 ? 8 : 4; rndColors = true; useFwdTrans = false;
            noiseScale = w2 ? 1.0 : 2.0; turbMult = .4; colorScale = 25.0; colorMult = w2 ? .3 : .2;
            pdMult = w2 ? d3(TWO_PI_F * 3.5, 7.9, 6.2) : d3(TWO_PI_F * 2.7, 3.6, 4.3);
          }
        } else if (c == "noise_color") {  // setTxtrColor (myScene.java:604-640)
          if (!useCustClrs) { useCustClrs = true; noiseColors.clear(); }
          Clr col;
          if (t.at(1) == "named") {
            if (!named_color(t.at(2), col)) { err = "unknown colour name: " + t.at(2); return false; }
          } else {
            col = clr(num(t, 1), num(t, 2), num(t, 3));
          }
          noiseColors.push_back(col);
        } else if (c == "stone") {  // setTexture (myScene.java:756-771): myCellularTexture
          reset_dflt_txtr();
          txtrType = RT_TEX_STONE;
          bool dflt = read_worley(t);
          if (!useCustClrs)
            noiseColors = {clr(0.2, 0.2, 0.2), clr(0.7, 0.7, 0.7), clr(0.6, 0.18, 0.22), clr(0.8, 0.26, 0.33),
                           clr(0.6, 0.32, 0.16), clr(0.8, 0.45, 0.25), clr(0.3, 0.01, 0.07), clr(0.6, 0.02, 0.13),
                           clr(0.4, 0.1, 0.17), clr(0.6, 0.3, 0.13)};  // clr_mortar1/2, clr_brick1_1 .. clr_brick4_2
          if (dflt) {
            octaves = 8; numPtsDist = 2; distFunc = 1; roiFunc = 1; rndColors = true; useFwdTrans = false;
            noiseScale = 4.0; turbMult = 1.0; colorScale = 12.0; colorMult = .2; avgNumPerCell = 1.0; mortarThresh = 0.05;
            pdMult = d3(10.0, 10.0, 10.0);
          }
        } else if (c == "begin") {  // :290-295
          poly = new_prim((t.size() > 1 && t[1] == "quad") ? RT_PRIM_QUAD : RT_PRIM_TRIANGLE);
          poly.nverts = poly.type == RT_PRIM_QUAD ? 4 : 3;
          inPoly = true;
          vc = 0;
        } else if (c == "texture_coord") {
          if (!inPoly || vc >= poly.nverts) throw std::out_of_range("texture_coord outside polygon");
          poly.uv[vc][0] = num(t, 1); poly.uv[vc][1] = num(t, 2);
        } else if (c == "vertex") {
          if (!inPoly || vc >= poly.nverts) throw std::out_of_range("vertex outside polygon");
          poly.v[vc][0] = num(t, 1); poly.v[vc][1] = num(t, 2); poly.v[vc][2] = num(t, 3);
          vc++;
        } else if (c == "end") {
          if (!inPoly) throw std::out_of_range("end without begin");
          add_prim(poly);
          inPoly = false;
        } else if (c == "sphere" || c == "sphereIn" || c == "moving_sphere" || c == "ellipsoid") {
          rt_prim_desc p = new_prim(c == "moving_sphere" ? RT_PRIM_MOVING_SPHERE : RT_PRIM_SPHERE);
          if (c == "ellipsoid") {
            p.p[3] = num(t, 1); p.p[4] = num(t, 2); p.p[5] = num(t, 3);
            p.p[0] = num(t, 4); p.p[1] = num(t, 5); p.p[2] = num(t, 6);
          } else {
            p.p[3] = p.p[4] = p.p[5] = num(t, 1);
            p.p[0] = num(t, 2); p.p[1] = num(t, 3); p.p[2] = num(t, 4);
          }
          if (c == "moving_sphere") { p.p[6] = num(t, 5); p.p[7] = num(t, 6); p.p[8] = num(t, 7); }
          if (c == "sphereIn") p.flags |= RT_PRIM_INVERTED;
          add_prim(p);
        } else if (c == "cyl" || c == "cylinder" || c == "hollow_cylinder") {
          rt_prim_desc p = new_prim(c == "hollow_cylinder" ? RT_PRIM_HOLLOW_CYLINDER : RT_PRIM_CYLINDER);
          double ox = 0, oy = 1, oz = 0;
          if (c == "cyl") {
            p.p[0] = num(t, 1); p.p[1] = num(t, 2); p.p[2] = num(t, 3); p.p[3] = num(t, 4); p.p[4] = num(t, 5);
            if (t.size() > 8) { ox = num(t, 6); oy = num(t, 7); oz = num(t, 8); }
          } else {  // cylinder radius x z ymin ymax
            p.p[0] = num(t, 1); p.p[2] = num(t, 2); p.p[4] = num(t, 3); p.p[3] = num(t, 4);
            p.p[1] = num(t, 5) - p.p[3];
          }
          p.p[5] = ox; p.p[6] = oy; p.p[7] = oz;
          add_prim(p);
        } else if (c == "box") {
          rt_prim_desc p = new_prim(RT_PRIM_BOX);
          for (int i = 0; i < 6; ++i) p.p[i] = num(t, 1 + i);
          add_prim(p);
        } else if (c == "plane") {
          rt_prim_desc p = new_prim(RT_PRIM_PLANE);
          for (int i = 0; i < 4; ++i) p.p[i] = num(t, 1 + i);
          p.nverts = 4;
          add_prim(p);
        } else if (c == "push") {
          push();
        } else if (c == "pop") {
          pop();
        } else if (c == "translate") {
          translate(num(t, 1), num(t, 2), num(t, 3));
        } else if (c == "scale") {
          scale(num(t, 1), num(t, 2), num(t, 3));
        } else if (c == "rotate") {
          rotate(num(t, 1), num(t, 2), num(t, 3), num(t, 4));
        } else if (c == "refine") {  // myScene.setRefine (myScene.java:796-803): progressive passes
          std::string v = t.at(1);
          for (auto& ch : v) ch = (char)std::tolower(ch);
          refine = v == "on" ? 1 : 0;
        } else if (c == "reset_timer" || c == "print_timer") {
          // timers are outside the kernel path
        } else {  // readRTFile's default case (myRTFileReader.java:343-345): report and go on
          std::fprintf(stderr, "When reading %s unknown command encountered : '%s' on line : [%d] : %s\n", fname.c_str(),
                       c.c_str(), lineNo, line.c_str());
          ++ignored;
        }
      } catch (const std::exception& e) {
        err = "parse error in " + fname + " at '" + c + "': " + e.what();
        return false;
      }
    }
    return true;
  }
};

}  // namespace

}  // namespace rt

using namespace rt;

static int load_desc(const char* scene_dir, const char* cli_file, int num_textures, const char* const* texture_names,
                     const rt_texture_desc* textures, CliLoader& L) {
  if (!scene_dir || !cli_file || (num_textures > 0 && (!texture_names || !textures)))
    return set_error(RT_E_INVALID, "rt_scene_load_cli: null argument");
  L.dir = scene_dir;
  std::memset(&L.d, 0, sizeof(L.d));
  L.d.fov = 60;  // default FOV scene (myRTFileReader.java:27-28)
  L.d.bkg_texture = -1;
  for (int i = 0; i < num_textures; ++i) L.texIndex[texture_names[i]] = i;
  if (!L.read(cli_file, true)) {
    bool io = L.err.rfind("cannot open", 0) == 0;
    return set_error(io ? RT_E_IO : RT_E_PARSE, L.err);
  }
  rt_scene_desc& d = L.d;
  d.num_prims = (int)L.prims.size(); d.prims = L.prims.data();
  d.num_materials = (int)L.mats.size(); d.materials = L.mats.data();
  d.num_lights = (int)L.lights.size(); d.lights = L.lights.data();
  d.num_accels = (int)L.accels.size(); d.accels = L.accels.data(); d.accel_members = L.members.data();
  d.num_top = (int)L.top.size(); d.top = L.top.data();
  d.num_instances = (int)L.insts.size(); d.instances = L.insts.data();
  d.num_textures = num_textures; d.textures = textures;
  return RT_OK;
}

extern "C" int rt_scene_load_cli(const char* scene_dir, const char* cli_file, int num_textures,
                                 const char* const* texture_names, const rt_texture_desc* textures, int device,
                                 rt_scene** out) {
  if (!out) return set_error(RT_E_INVALID, "rt_scene_load_cli: null out");
  CliLoader L;
  int rc = load_desc(scene_dir, cli_file, num_textures, texture_names, textures, L);
  if (rc) return rc;
  rc = rt_scene_create(&L.d, device, out);
  if (rc == RT_OK) (*out)->saveName = L.saveName.empty() ? std::string(cli_file) : L.saveName;
  if (rc == RT_OK) (*out)->refine = L.refine == 1;
  return rc;
}

static int put_name(const std::string& n, char* buf, int cap) {
  if (buf && cap > (int)n.size()) std::memcpy(buf, n.c_str(), n.size() + 1);
  return (int)n.size();
}

// myScene.saveFile (myScene.java:1185-1196): saveName.split("\\.(?=[^\\.]+$)")[0] + ".png" --
// cut at the last '.' when at least one non-'.' character follows it (flipNormal's
// "_normFlipped" suffix is a UI action, not part of the render path).
extern "C" int rt_png_name(const char* save_name, char* buf, int cap) {
  if (!save_name) return set_error(RT_E_INVALID, "rt_png_name: null name");
  std::string n = save_name;
  size_t dot = n.rfind('.');
  if (dot != std::string::npos && dot + 1 < n.size()) n.resize(dot);
  return put_name(n + ".png", buf, cap);
}

extern "C" int rt_scene_save_name(const rt_scene* s, char* buf, int cap) {
  if (!s) return set_error(RT_E_INVALID, "rt_scene_save_name: null scene");
  if (s->saveName.empty()) return set_error(RT_E_INVALID, "rt_scene_save_name: scene not loaded from a .cli");
  return rt_png_name(s->saveName.c_str(), buf, cap);
}

// Host-only: parse + build the flattened scene without touching a device, report the
// rt_scene_info fields (device bytes = host layout bytes). Used by the CPU test suite.
extern "C" int rt_scene_inspect_cli(const char* scene_dir, const char* cli_file, int num_textures,
                                    const char* const* texture_names, const rt_texture_desc* textures, int64_t* info,
                                    int n) {
  if (!info) return set_error(RT_E_INVALID, "null info");
  CliLoader L;
  int rc = load_desc(scene_dir, cli_file, num_textures, texture_names, textures, L);
  if (rc) return rc;
  HostScene hs;
  rc = build_host_scene(&L.d, hs);
  if (rc) return rc;
  int64_t bytes = (int64_t)(hs.xf.size() * sizeof(XformD) + hs.tri.size() * (sizeof(TriD) + sizeof(TriF)) + hs.prim.size() * sizeof(PrimD) +
                            hs.node.size() * (sizeof(NodeD) + sizeof(NodeF)) + hs.leaf.size() * sizeof(LeafD) + hs.member.size() * 4 +
                            hs.accel.size() * sizeof(AccelD) + hs.top.size() * sizeof(TopD) + hs.mat.size() * sizeof(MatD) +
                            hs.light.size() * sizeof(LightD) + hs.texel.size() * 4);
  int64_t v[14] = {(int64_t)hs.top.size(), (int64_t)hs.light.size(), hs.bvhInternal, hs.bvhLeaves, hs.bvhDepth,
                   hs.bvhPrims, hs.nprims, hs.rpp, bytes, (int64_t)hs.tri.size(), 0, (int64_t)hs.mat.size(),
                   hs.photonMode, hs.photonCount};
  for (int i = 0; i < n && i < 14; ++i) info[i] = v[i];
  return RT_OK;
}
