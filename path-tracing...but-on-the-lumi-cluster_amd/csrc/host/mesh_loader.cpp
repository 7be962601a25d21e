// OBJ/MTL loading - restatement of load_mesh / load_mtl (mesh.cc:10-265).
//
// Produces the same vertex/index arrays as the reference: vertices are the
// distinct (position, texcoord, normal, material) index groups in order of
// first appearance (mesh.cc:216-262), per-vertex material = (Pr, Pm,
// max(Tf), max(scaled Ke)) and albedo = (Kd, d).  Parsing uses the same
// strtof / strtol(base 0) conversions so every float is bit-identical.
#include "scene_internal.h"
#include "hmath.h"
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <unordered_map>

namespace ptg {
namespace {

using namespace hm;

struct Material {                       // mtl_material, mesh.cc:10-19
    std::string name;
    f3 albedo = v3(1, 1, 1);
    float alpha = 0;
    f3 emission = v3(0, 0, 0);
    float roughness = 1;
    float metallicness = 0;
    f3 transmission = v3(0, 0, 0);
};

std::vector<char> slurp(const std::string& path)
{
    FILE* f = fopen(path.c_str(), "rb");
    if(!f) throw std::runtime_error("Unable to open " + path);
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<char> buf(size_t(n) + 1);
    size_t got = n > 0 ? fread(buf.data(), 1, size_t(n), f) : 0;
    fclose(f);
    if(got != size_t(n)) throw std::runtime_error("Unable to read " + path);
    buf[size_t(n)] = 0;
    return buf;
}

// A cursor over a NUL-terminated file image with the reference's tokenizer
// rules: a keyword is the run of non-space characters after leading
// whitespace, and it "matches" a name when strncmp over the keyword's own
// length agrees (mesh.cc:71-73, 160-162).
struct Cursor {
    char* p;
    bool at_end() const { return *p == 0; }
    void skip_space() { while(isspace((unsigned char)*p)) ++p; }
    std::pair<const char*, int> keyword()
    {
        skip_space();
        const char* k = p;
        int n = 0;
        while(*p && !isspace((unsigned char)*p)) { ++p; ++n; }
        return {k, n};
    }
    static bool is(std::pair<const char*, int> kw, const char* name) { return strncmp(kw.first, name, kw.second) == 0; }
    float real() { return strtof(p, &p); }
    long integer() { return strtol(p, &p, 0); }
    std::string word()
    {
        skip_space();
        const char* s = p;
        while(*p && !isspace((unsigned char)*p)) ++p;
        return std::string(s, p - s);
    }
    void next_line() { while(*p && *p != '\n') ++p; }
};

void read_mtl(std::vector<Material>& mats, const std::string& path)
{
    std::vector<char> text = slurp(path);
    Cursor c{text.data()};
    Material* cur = nullptr;
    while(!c.at_end())
    {
        auto kw = c.keyword();
        if(Cursor::is(kw, "newmtl"))
        {
            Material m;
            m.name = c.word();
            mats.push_back(m);
            cur = &mats.back();
        }
        else if(cur)
        {
            if(Cursor::is(kw, "Kd")) { cur->albedo.x = c.real(); cur->albedo.y = c.real(); cur->albedo.z = c.real(); }
            else if(Cursor::is(kw, "Ke")) { cur->emission.x = c.real(); cur->emission.y = c.real(); cur->emission.z = c.real(); }
            else if(Cursor::is(kw, "d")) cur->alpha = c.real();
            else if(Cursor::is(kw, "Pr")) cur->roughness = c.real();
            else if(Cursor::is(kw, "Pm")) cur->metallicness = c.real();
            else if(Cursor::is(kw, "Tf"))
            { cur->transmission.x = c.real(); cur->transmission.y = c.real(); cur->transmission.z = c.real(); }
        }
        c.next_line();
    }
}

struct Corner {                         // index_group, mesh.cc:118-137
    int pos = -1, tex = -1, normal = -1, material = -1;
    bool operator==(const Corner& o) const
    { return pos == o.pos && tex == o.tex && normal == o.normal && material == o.material; }
};
struct CornerHash {
    size_t operator()(const Corner& k) const
    {
        uint64_t h = uint64_t(uint32_t(k.pos)) * 0x9E3779B97F4A7C15ull;
        h ^= (uint64_t(uint32_t(k.tex)) + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2));
        h ^= (uint64_t(uint32_t(k.normal)) * 0xC2B2AE3D27D4EB4Full + (h << 6) + (h >> 2));
        h ^= (uint64_t(uint32_t(k.material)) + 0x165667B19E3779F9ull + (h << 6) + (h >> 2));
        return size_t(h);
    }
};

} // namespace

ptg_mesh load_obj_mesh(MeshBuffers& mb, const std::string& obj_path)
{
    ptg_mesh m;
    m.index_offset = uint32_t(mb.indices.size());
    m.base_vertex_offset = uint32_t(mb.pos.size());

    std::vector<f3> positions, normals;
    std::vector<Material> mats(1);     // index 0: the default material
    std::vector<Corner> corners;
    size_t ntex = 0;
    int active = 0;
    const std::string dir = obj_path.substr(0, obj_path.rfind('/') + 1);

    std::vector<char> text = slurp(obj_path);
    Cursor c{text.data()};
    while(!c.at_end())
    {
        auto kw = c.keyword();
        if(Cursor::is(kw, "v"))
        {
            f3 p;
            p.x = c.real(); p.y = c.real(); p.z = c.real();
            positions.push_back(p);
        }
        else if(Cursor::is(kw, "vn"))
        {
            f3 n;
            n.x = c.real(); n.y = c.real(); n.z = c.real();
            normals.push_back(normalize(n));
        }
        else if(Cursor::is(kw, "vt"))
        {
            c.real(); c.real();
            ++ntex;
        }
        else if(Cursor::is(kw, "f"))
        {
            for(int k = 0; k < 3; ++k)
            {
                Corner g;
                g.material = active;
                g.pos = int(c.integer() - 1);
                if(*c.p == '/') ++c.p;
                g.tex = int(c.integer() - 1);
                if(*c.p == '/') ++c.p;
                g.normal = int(c.integer() - 1);
                corners.push_back(g);
            }
        }
        else if(Cursor::is(kw, "usemtl"))
        {
            std::string name = c.word();
            for(size_t i = 0; i < mats.size(); ++i)
                if(mats[i].name == name) { active = int(i); break; }
        }
        else if(Cursor::is(kw, "mtllib"))
            read_mtl(mats, dir + c.word());
        c.next_line();
    }

    m.triangle_count = uint32_t(corners.size() / 3);
    m.vertex_count = 0;
    std::unordered_map<Corner, uint32_t, CornerHash> first_seen;
    first_seen.reserve(corners.size());
    mb.indices.reserve(mb.indices.size() + corners.size());
    for(const Corner& g: corners)
    {
        auto it = first_seen.find(g);
        if(it == first_seen.end())
        {
            it = first_seen.emplace(g, uint32_t(first_seen.size())).first;
            f3 p = v3(0, 0, 0), n = v3(0, 0, 0);
            if(g.pos >= 0 && size_t(g.pos) < positions.size()) p = positions[g.pos];
            if(g.normal >= 0 && size_t(g.normal) < normals.size()) n = normals[g.normal];
            f4 albedo = v4(0, 0, 0, 0), material = v4(0, 0, 0, 0);
            if(g.material >= 0 && size_t(g.material) < mats.size())
            {
                const Material& mt = mats[g.material];
                albedo = v4(mt.albedo.x, mt.albedo.y, mt.albedo.z, mt.alpha);
                material.x = mt.roughness;
                material.y = mt.metallicness;
                // emission relative to the brighter of albedo / emission (mesh.cc:243-249)
                f3 se = vmax(mt.emission / vmax(mt.albedo, mt.emission), v3(0, 0, 0));
                if(mt.emission.x == 0) se.x = 0;
                if(mt.emission.y == 0) se.y = 0;
                if(mt.emission.z == 0) se.z = 0;
                material.z = fmaxf_(mt.transmission.x, fmaxf_(mt.transmission.y, mt.transmission.z));
                material.w = fmaxf_(se.x, fmaxf_(se.y, se.z));
            }
            mb.pos.push_back(p);
            mb.normal.push_back(n);
            mb.albedo.push_back(albedo);
            mb.material.push_back(material);
            m.vertex_count++;
        }
        mb.indices.push_back(it->second);
    }
    (void)ntex;
    return m;
}

} // namespace ptg
