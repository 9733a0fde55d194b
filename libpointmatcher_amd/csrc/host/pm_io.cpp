// pm_io.cpp — DataPoints::load for the CSV and VTK formats (IO.cpp:374-389,
// loadCSV :535-800, loadVTK :918-1252), the clouds either side of the ICP.
//
// Same label mapping as the reference: the supported external names
// (IO.h:117-161: x y z pad, nx ny nz / normal_x.., observationDirections0..2,
// red green blue alpha, eigValues0..2, eigVectors<0-2><X-Z>, intensity) are
// collected in that table's order into feature / descriptor labels (a repeated
// internal name grows its span); every other column becomes a descriptor of
// its own name, in file order; a missing "pad" row is added as ones.  VTK:
// POINTS (float / double, ASCII or big-endian BINARY) with the homogeneous
// row, POLYDATA / UNSTRUCTURED_GRID cell blocks skipped, POINT_DATA
// SCALARS / VECTORS / NORMALS / TENSORS / COLOR_SCALARS and FIELD arrays as
// descriptors.  Departures (documented in DESIGN.md): time columns / split
// time fields are dropped (this DataPoints carries no times); a header-less
// CSV with other than 2 or 3 columns is an error (the reference prompts on
// stdin for the x / y / z columns); the CSV body is parsed on several host
// threads.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "pm_icp.h"

namespace pm {

namespace {

enum PropType { kFeature, kDescriptor, kTime, kUnsupported };
struct SupLabel {
    const char* internal;
    const char* external;
    PropType type;
};
const SupLabel kLabels[] = {
    {"x", "x", kFeature}, {"y", "y", kFeature}, {"z", "z", kFeature}, {"pad", "pad", kFeature},
    {"normals", "nx", kDescriptor}, {"normals", "ny", kDescriptor}, {"normals", "nz", kDescriptor},
    {"normals", "normal_x", kDescriptor}, {"normals", "normal_y", kDescriptor}, {"normals", "normal_z", kDescriptor},
    {"observationDirections", "observationDirections0", kDescriptor},
    {"observationDirections", "observationDirections1", kDescriptor},
    {"observationDirections", "observationDirections2", kDescriptor},
    {"color", "red", kDescriptor}, {"color", "green", kDescriptor}, {"color", "blue", kDescriptor},
    {"color", "alpha", kDescriptor},
    {"eigValues", "eigValues0", kDescriptor}, {"eigValues", "eigValues1", kDescriptor},
    {"eigValues", "eigValues2", kDescriptor},
    {"eigVectors", "eigVectors0X", kDescriptor}, {"eigVectors", "eigVectors0Y", kDescriptor},
    {"eigVectors", "eigVectors0Z", kDescriptor}, {"eigVectors", "eigVectors1X", kDescriptor},
    {"eigVectors", "eigVectors1Y", kDescriptor}, {"eigVectors", "eigVectors1Z", kDescriptor},
    {"eigVectors", "eigVectors2X", kDescriptor}, {"eigVectors", "eigVectors2Y", kDescriptor},
    {"eigVectors", "eigVectors2Z", kDescriptor},
    {"intensity", "intensity", kDescriptor},
    {"time", "time", kTime},
};

// LabelGenerator::add (IO.cpp:427-446): a repeated name grows its span
void label_add(std::vector<std::pair<std::string, int>>& ls, const std::string& name) {
    for (auto& l : ls)
        if (l.first == name) {
            ++l.second;
            return;
        }
    ls.push_back({name, 1});
}

// safeGetLine (IO.cpp): \n, \r\n or \r line ends
bool get_line(std::istream& is, std::string& line) {
    line.clear();
    std::istream::sentry se(is, true);
    std::streambuf* sb = is.rdbuf();
    for (;;) {
        const int c = sb->sbumpc();
        switch (c) {
        case '\n': return true;
        case '\r':
            if (sb->sgetc() == '\n') sb->sbumpc();
            return true;
        case std::streambuf::traits_type::eof():
            if (line.empty()) is.setstate(std::ios::eofbit);
            return !line.empty();
        default: line += (char)c;
        }
    }
}

std::vector<std::string> tokens(const std::string& line) {
    std::vector<std::string> out;
    const char* delim = " \t,;";
    size_t i = 0;
    while (i < line.size()) {
        i = line.find_first_not_of(delim, i);
        if (i == std::string::npos) break;
        const size_t j = line.find_first_of(delim, i);
        out.push_back(line.substr(i, j == std::string::npos ? std::string::npos : j - i));
        i = j == std::string::npos ? line.size() : j;
    }
    return out;
}

// lexical_cast<T>: parsed straight into T (strtof for float: one rounding)
template <typename T>
T parse_scalar(const std::string& s, bool& ok) {
    char* end = nullptr;
    const T v = sizeof(T) == 4 ? (T)std::strtof(s.c_str(), &end) : (T)std::strtod(s.c_str(), &end);
    ok = end && *end == '\0' && end != s.c_str();
    return v;
}

template <typename T>
void assemble(DataPoints<T>& dp, int64_t n, const std::vector<std::pair<std::string, int>>& fl,
              const std::vector<std::vector<T>>& frows, const std::vector<std::pair<std::string, int>>& dl,
              const std::vector<std::vector<T>>& drows) {
    // every row holds exactly n values (a malformed file must not make the
    // copies below read past a row)
    for (const auto& r : frows)
        if ((int64_t)r.size() != n) throw std::runtime_error("cloud parse error: a feature row does not hold every point");
    for (const auto& r : drows)
        if ((int64_t)r.size() != n) throw std::runtime_error("cloud parse error: a descriptor row does not hold every point");
    bool has_pad = false;
    for (auto& l : fl) has_pad = has_pad || l.first == "pad";
    const int fdim = (int)frows.size() + (has_pad ? 0 : 1);
    dp.n = n;
    dp.rows = fdim;
    dp.features.assign((size_t)(n * fdim), (T)1);
    for (int64_t i = 0; i < n; ++i)
        for (size_t r = 0; r < frows.size(); ++r) dp.features[(size_t)(i * fdim + (int64_t)r)] = frows[r][(size_t)i];
    dp.featureLabels.clear();
    for (auto& l : fl) dp.featureLabels.push_back({l.first, l.second});
    if (!has_pad) dp.featureLabels.push_back({"pad", 1});  // (IO.cpp:792-796)
    dp.descDim = (int)drows.size();
    dp.descriptors.assign((size_t)(n * dp.descDim), (T)0);
    for (int64_t i = 0; i < n; ++i)
        for (int r = 0; r < dp.descDim; ++r) dp.descriptors[(size_t)(i * dp.descDim + r)] = drows[(size_t)r][(size_t)i];
    dp.descriptorLabels.clear();
    for (auto& l : dl) dp.descriptorLabels.push_back({l.first, l.second});
}

}  // namespace

// PointMatcherIO::loadCSV (IO.cpp:535-800)
template <typename T>
DataPoints<T> load_csv(std::istream& is) {
    std::vector<std::string> lines;
    std::string line;
    while (get_line(is, line)) {
        if (line.empty()) break;  // (an empty line ends the data, :567-568)
        lines.push_back(line);
    }
    DataPoints<T> dp;
    if (lines.empty()) {
        assemble<T>(dp, 0, {}, {}, {}, {});
        return dp;
    }
    // header: any character outside " ,+-.1234567890Ee" (:571-580)
    const bool header = std::strspn(lines[0].c_str(), " ,+-.1234567890Ee") != lines[0].size();
    std::vector<std::string> names = tokens(lines[0]);
    if (!header) {
        const size_t dim = names.size();
        if (dim != 2 && dim != 3)
            throw std::runtime_error("CSV parse error: " + std::to_string(dim) +
                                     " columns and no header: not obvious which columns to load for x, y or z");
        names = dim == 2 ? std::vector<std::string>{"x", "y"} : std::vector<std::string>{"x", "y", "z"};
    }
    const size_t ncol = names.size();
    std::vector<PropType> ctype(ncol, kUnsupported);
    std::vector<int> crow(ncol, 0);
    std::vector<std::pair<std::string, int>> fl, dl, tl;
    int nf = 0, nd = 0, nt = 0;
    for (const SupLabel& s : kLabels)  // (:655-693, the table's order)
        for (size_t j = 0; j < ncol; ++j)
            if (names[j] == s.external) {
                ctype[j] = s.type;
                if (s.type == kFeature) {
                    crow[j] = nf++;
                    label_add(fl, s.internal);
                } else if (s.type == kDescriptor) {
                    crow[j] = nd++;
                    label_add(dl, s.internal);
                } else {
                    crow[j] = nt++;
                    label_add(tl, s.internal);
                }
                break;
            }
    for (size_t j = 0; j < ncol; ++j)  // unsupported: descriptors of their own name (:696-705)
        if (ctype[j] == kUnsupported) {
            ctype[j] = kDescriptor;
            crow[j] = nd++;
            label_add(dl, names[j]);
        }
    const size_t first = header ? 1 : 0;
    const int64_t n = (int64_t)(lines.size() - first);
    std::vector<std::vector<T>> frows((size_t)nf, std::vector<T>((size_t)n)), drows((size_t)nd,
                                                                                       std::vector<T>((size_t)n));
    // the body, on several threads (each line is independent)
    std::vector<std::string> errs;
    const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(8, n / 20000));
    std::vector<std::string> terr((size_t)nth);
    auto work = [&](int t) {
        for (int64_t i = t; i < n; i += nth) {
            const std::vector<std::string> tk = tokens(lines[first + (size_t)i]);
            if (tk.size() > ncol) {
                terr[(size_t)t] = "CSV parse error: at line " + std::to_string(i) +
                                  ", too many elements to parse compare to the header number of columns (col=" +
                                  std::to_string(ncol) + ").";
                return;
            }
            if (tk.size() < ncol) {
                terr[(size_t)t] = "CSV parse error: at line " + std::to_string(i) +
                                  ", not enough elements to parse compare to the header number of columns (col=" +
                                  std::to_string(ncol) + ").";
                return;
            }
            for (size_t j = 0; j < ncol; ++j) {
                if (ctype[j] == kTime) continue;  // (times dropped: no time matrix here)
                bool ok = true;
                const T v = parse_scalar<T>(tk[j], ok);
                if (!ok) {
                    terr[(size_t)t] = "CSV parse error: at line " + std::to_string(i) + ", cannot convert '" + tk[j] + "'";
                    return;
                }
                (ctype[j] == kFeature ? frows : drows)[(size_t)crow[j]][(size_t)i] = v;
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (auto& e : terr)
        if (!e.empty()) throw std::runtime_error(e);
    assemble<T>(dp, n, fl, frows, dl, drows);
    return dp;
}

namespace {

template <typename T, typename S>
void read_values(std::istream& is, bool binary, int64_t count, std::vector<T>& out) {
    out.resize((size_t)count);
    for (int64_t i = 0; i < count; ++i) {
        if (binary) {  // big-endian (IOFunctions.h:108-133)
            unsigned char b[sizeof(S)];
            is.read((char*)b, sizeof(S));
            std::reverse(b, b + sizeof(S));
            S v;
            std::memcpy(&v, b, sizeof(S));
            out[(size_t)i] = (T)v;
        } else {
            T v;  // (istream >> T, as the reference's `in >> dest`)
            is >> v;
            out[(size_t)i] = v;
        }
        if (!is) throw std::runtime_error("VTK parse error: truncated data");
    }
}
template <typename T>
void read_typed(std::istream& is, bool binary, const std::string& type, int64_t count, std::vector<T>& out) {
    if (type == "float")
        read_values<T, float>(is, binary, count, out);
    else if (type == "double")
        read_values<T, double>(is, binary, count, out);
    else if (type == "unsigned_int")
        read_values<T, unsigned int>(is, binary, count, out);
    else
        throw std::runtime_error("VTK parse error: data type " + type + " can only be float or double");
}

void skip_block(bool binary, int bsize, std::istream& is, bool separate_size = true) {  // skipBlock (:918-946)
    long long n = 0, size = 0;
    is >> n;
    if (!is.good()) throw std::runtime_error("File violates the VTK format : parameter 'n' is missing after a field name.");
    if (separate_size) {
        is >> size;
        if (!is.good())
            throw std::runtime_error("File violates the VTK format : parameter 'size' is missing after a field name.");
    } else {
        size = n;
    }
    std::string line;
    get_line(is, line);
    if (binary) {
        is.seekg(size * bsize, std::ios_base::cur);
    } else {
        for (long long p = 0; p < n; ++p) get_line(is, line);
    }
}

}  // namespace

// PointMatcherIO::loadVTK (IO.cpp:948-1252)
template <typename T>
DataPoints<T> load_vtk(std::istream& is) {
    std::string line;
    get_line(is, line);
    if (line.find("# vtk DataFile Version") != 0) throw std::runtime_error("Wrong magic header, found " + line);
    get_line(is, line);
    get_line(is, line);
    const bool binary = line == "BINARY";
    if (line != "ASCII" && !binary) throw std::runtime_error("Wrong file type, expecting ASCII or BINARY, found " + line);
    get_line(is, line);
    bool poly;
    if (line == "DATASET POLYDATA")
        poly = true;
    else if (line == "DATASET UNSTRUCTURED_GRID")
        poly = false;
    else
        throw std::runtime_error("Wrong data type, expecting DATASET POLYDATA, found " + line);
    int64_t count = 0;
    bool have_points = false;
    std::vector<T> pts;
    std::vector<std::pair<std::string, int>> dl;
    std::vector<std::vector<T>> drows;
    auto add_desc = [&](const std::string& name, int dim, const std::vector<T>& v) {  // v: count x dim point-major
        if ((int64_t)v.size() != count * (int64_t)dim)
            throw std::runtime_error("VTK parse error: descriptor " + name + " does not hold every point");
        dl.push_back({name, dim});
        for (int r = 0; r < dim; ++r) {
            std::vector<T> row((size_t)count);
            for (int64_t i = 0; i < count; ++i) row[(size_t)i] = v[(size_t)(i * dim + r)];
            drows.push_back(std::move(row));
        }
    };
    std::string field;
    while (is >> field) {
        if (field == "POINTS") {
            std::string type;
            if (have_points) throw std::runtime_error("VTK parse error: a second POINTS block");
            is >> count >> type;
            if (!is || count < 0) throw std::runtime_error("VTK parse error: bad POINTS count");
            have_points = true;
            get_line(is, line);
            if (type != "float" && type != "double") throw std::runtime_error("Field POINTS can only be of type double or float");
            read_typed<T>(is, binary, type, count * 3, pts);
        } else if (poly && (field == "VERTICES" || field == "LINES" || field == "POLYGONS" || field == "TRIANGLE_STRIPS")) {
            skip_block(binary, 4, is);
        } else if (!poly && field == "CELLS") {
            skip_block(binary, 4, is);
        } else if (!poly && field == "CELL_TYPES") {
            skip_block(binary, 4, is, false);
        } else if (field == "POINT_DATA") {
            int64_t c = 0;
            is >> c;
            if (c != count) throw std::runtime_error("The size of POINTS is different than POINT_DATA");
        } else if (field == "FIELD") {
            std::string fname;
            int nfield = 0;
            is >> fname >> nfield;
            if (!is || nfield < 0) throw std::runtime_error("VTK parse error: bad FIELD header");
            for (int f = 0; f < nfield; ++f) {
                std::string name, type;
                int dim = 0;
                int64_t tuples = 0;
                is >> name >> dim >> tuples >> type;
                if (!is || dim < 0 || tuples < 0) throw std::runtime_error("VTK parse error: bad FIELD array " + name);
                if (type == "vtkIdType") {  // skipped
                    if (binary) {
                        is.seekg(dim * tuples * 4, std::ios_base::cur);
                    } else {
                        long long t;
                        for (int64_t k = 0; k < dim * tuples; ++k) is >> t;
                    }
                    continue;
                }
                if (type != "float" && type != "double")
                    throw std::runtime_error("Field FIELD is " + type + " but can only be of type double or float");
                // (point data: the reference reads pointCount tuples, IO.cpp:1082-1083;
                // a dataset-level array before POINTS has no point count to read)
                if (!have_points) throw std::runtime_error("VTK parse error: FIELD array " + name + " before POINTS");
                std::vector<T> v;
                read_typed<T>(is, binary, type, count * dim, v);
                add_desc(name, dim, v);
            }
        } else if (field == "METADATA") {
            get_line(is, line);
            get_line(is, line);
            while (!line.empty()) get_line(is, line);
        } else {
            std::string name, type;
            is >> name;
            auto ends = [&](const std::string& suf) {
                return name.size() >= suf.size() && name.compare(name.size() - suf.size(), suf.size(), suf) == 0;
            };
            const bool time_part = ends("_splitTime_high32") || ends("_splitTime_low32");
            int dim = 0;
            bool lookup = false, color = false;
            if (field == "SCALARS") {
                dim = 1;
                is >> type;
                lookup = true;
            } else if (field == "VECTORS" || field == "NORMALS") {
                dim = 3;
                is >> type;
            } else if (field == "TENSORS") {
                dim = 9;
                is >> type;
            } else if (field == "COLOR_SCALARS") {
                is >> dim;
                type = "float";
                color = true;
            } else {
                throw std::runtime_error("Unknown field name " + field +
                                         ", expecting SCALARS, VECTORS, TENSORS, NORMALS or COLOR_SCALARS.");
            }
            if (!have_points) throw std::runtime_error("VTK parse error: " + field + " " + name + " before POINTS");
            if (dim < 0 || dim > 4096) throw std::runtime_error("VTK parse error: bad COLOR_SCALARS dimension");
            get_line(is, line);
            std::vector<T> v;
            if (color && binary) {  // unsigned char / 255 (:1195-1204)
                v.resize((size_t)(count * dim));
                std::vector<unsigned char> b((size_t)dim);
                for (int64_t i = 0; i < count; ++i) {
                    is.read((char*)b.data(), dim);
                    for (int r = 0; r < dim; ++r) v[(size_t)(i * dim + r)] = (T)b[(size_t)r] / (T)255.0;
                }
            } else {
                if (lookup) get_line(is, line);  // LOOKUP_TABLE
                read_typed<T>(is, binary, time_part ? std::string("unsigned_int") : type, count * dim, v);
            }
            if (!time_part) add_desc(name, dim, v);  // (split times dropped: no time matrix here)
        }
    }
    std::vector<std::pair<std::string, int>> fl = {{"x", 1}, {"y", 1}, {"z", 1}, {"pad", 1}};
    std::vector<std::vector<T>> frows(4, std::vector<T>((size_t)count, (T)1));
    for (int64_t i = 0; i < count && !pts.empty(); ++i)
        for (int r = 0; r < 3; ++r) frows[(size_t)r][(size_t)i] = pts[(size_t)(i * 3 + r)];
    DataPoints<T> dp;
    assemble<T>(dp, count, pts.empty() ? std::vector<std::pair<std::string, int>>{} : fl,
                pts.empty() ? std::vector<std::vector<T>>{} : frows, dl, drows);
    return dp;
}

// DataPoints::load (IO.cpp:374-389): by extension
template <typename T>
DataPoints<T> load_cloud(const std::string& path) {
    std::string ext = path.size() >= 4 ? path.substr(path.size() - 4) : "";
    std::transform(ext.begin(), ext.end(), ext.begin(), ::tolower);
    if (ext == ".vtk" || ext == ".csv") {
        std::ifstream ifs(path.c_str(), std::ios::binary);
        if (!ifs.good()) throw std::runtime_error("Cannot open file " + path);  // (validateFile, IO.cpp:355-371)
        return ext == ".vtk" ? load_vtk<T>(ifs) : load_csv<T>(ifs);
    }
    throw std::runtime_error("DataPoints::load(): Unknown extension \"" + ext + "\" for file \"" + path +
                             "\", extension must be either \".vtk\" or \".csv\"");
}

template DataPoints<float> load_cloud<float>(const std::string&);
template DataPoints<double> load_cloud<double>(const std::string&);

}  // namespace pm
