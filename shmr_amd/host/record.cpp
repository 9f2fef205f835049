// Durable record of a VirtualFile: its block list with every block's
// BlockTopology and shard paths, in the shape the reference persists it.
//
// The reference keeps each inode's VirtualFile in the superblock (DataBunny:
// sled values written with serde_yaml::to_vec, read back with
// serde_yaml::from_slice -- src/databunny.rs:297-327, src/types.rs:17-29) via
// #[derive(Serialize, Deserialize)] on VirtualFile (src/vfs/mod.rs:35-56),
// VirtualBlock (src/vfs/block.rs:119-158, runtime fields #[serde(skip)]),
// BlockTopology (block.rs:22-30) and VirtualPath (src/vfs/path.rs:20-28).
// serde_yaml 0.9 writes an externally tagged enum as a YAML tag: the unit
// variant as `Single`, the newtype variant as `!Mirror 3`, the tuple variant
// as a tagged sequence (`!Erasure` then `- 1`, `- 8`, `- 3`), and sequences
// in mapping values without extra indentation.  This file writes that text
// and reads it back (also flow sequences such as `!Erasure [1, 8, 3]`), so a
// file rewritten to Erasure(1, k, p) reloads as Erasure blocks after a
// restart.  The sled store, zstd and the superblock entry around the record
// stay out of scope.  Byte equality with serde_yaml's
// own output is not pinned (no Rust toolchain here); the field names, order
// and enum encoding follow the derives above.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <unistd.h>

#include <fstream>
#include <sstream>

#include "vfs.hpp"

namespace shmr {

namespace {

// ---- emitter -----------------------------------------------------------------

bool looks_special(const std::string& s) {
    std::string l;
    for (char c : s) l += char(std::tolower(static_cast<unsigned char>(c)));
    static const char* kWords[] = {"~", "null", "true", "false", "yes", "no", "on", "off", "y", "n",
                                   ".inf", "-.inf", "+.inf", ".nan"};
    for (const char* w : kWords)
        if (l == w) return true;
    // numbers (decimal, hex, octal, floats): anything strtod / strtoll consume fully
    char* end = nullptr;
    errno = 0;
    (void)std::strtod(s.c_str(), &end);
    if (end && *end == '\0') return true;
    (void)std::strtoll(s.c_str(), &end, 0);
    return end && *end == '\0';
}

std::string yaml_str(const std::string& s) {
    bool plain = !s.empty() && !looks_special(s) && s.front() != ' ' && s.back() != ' ' && s.back() != ':';
    if (plain && std::strchr("-?:,[]{}#&*!|>'\"%@`", s.front())) plain = false;
    if (plain && (s.find(": ") != std::string::npos || s.find(" #") != std::string::npos)) plain = false;
    bool control = false;
    for (unsigned char c : s)
        if (c < 0x20 || c == 0x7f) control = true;
    if (plain && !control) return s;
    if (!control) {   // single-quoted, '' escapes a quote
        std::string q = "'";
        for (char c : s) q += (c == '\'') ? std::string("''") : std::string(1, c);
        return q + "'";
    }
    std::string q = "\"";   // double-quoted with escapes
    for (unsigned char c : s) {
        char buf[8];
        if (c == '"' || c == '\\') {
            q += '\\';
            q += char(c);
        } else if (c < 0x20 || c == 0x7f) {
            std::snprintf(buf, sizeof buf, "\\x%02x", c);
            q += buf;
        } else {
            q += char(c);
        }
    }
    return q + "\"";
}

void emit_block(std::ostringstream& o, const VirtualBlock& b) {
    o << "- ino: " << b.ino << "\n";
    o << "  idx: " << b.idx << "\n";
    o << "  size: " << b.size << "\n";
    switch (b.topology.kind) {
        case BlockTopology::Single: o << "  topology: Single\n"; break;
        case BlockTopology::Mirror: o << "  topology: !Mirror " << unsigned(b.topology.n) << "\n"; break;
        case BlockTopology::Erasure:
            o << "  topology: !Erasure\n  - " << unsigned(b.topology.version) << "\n  - " << unsigned(b.topology.data)
              << "\n  - " << unsigned(b.topology.parity) << "\n";
            break;
    }
    if (b.shards.empty()) {
        o << "  shards: []\n";
        return;
    }
    o << "  shards:\n";
    for (const auto& s : b.shards) {
        o << "  - pool: " << yaml_str(s.pool) << "\n";
        o << "    bucket: " << yaml_str(s.bucket) << "\n";
        o << "    filename: " << yaml_str(s.filename) << "\n";
    }
}

// ---- parser (the block/flow subset the emitter and serde_yaml produce) -------

struct Node {
    enum Kind { Scalar, Seq, Map } kind = Scalar;
    std::string tag;     // "!Erasure" ...
    std::string value;   // Scalar
    std::vector<Node> items;                             // Seq
    std::vector<std::pair<std::string, Node>> entries;   // Map
    const Node* get(const std::string& k) const {
        for (auto& e : entries)
            if (e.first == k) return &e.second;
        return nullptr;
    }
};

struct Line {
    int indent;
    std::string text;   // without indentation; comments and trailing blanks removed
};

struct ParseError {
    std::string what;
};

std::string strip_comment(const std::string& s) {
    // a '#' after whitespace outside quotes starts a comment
    char q = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (q) {
            if (q == '"' && c == '\\') ++i;   // escaped character inside "..."
            else if (c == q) q = 0;
            continue;
        }
        if (c == '\'' || c == '"') q = c;
        else if (c == '#' && (i == 0 || s[i - 1] == ' ')) return s.substr(0, i);
    }
    return s;
}

std::string rtrim(std::string s) {
    while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
    return s;
}

std::string unquote(const std::string& s) {
    if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
        std::string o;
        for (size_t i = 1; i + 1 < s.size(); ++i) {
            o += s[i];
            if (s[i] == '\'' && s[i + 1] == '\'') ++i;
        }
        return o;
    }
    if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
        std::string o;
        for (size_t i = 1; i + 1 < s.size(); ++i) {
            if (s[i] != '\\') {
                o += s[i];
                continue;
            }
            const char e = s[++i];
            if (e == 'n') o += '\n';
            else if (e == 't') o += '\t';
            else if (e == 'x' && i + 2 < s.size()) {
                o += char(std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
                i += 2;
            } else {
                o += e;
            }
        }
        return o;
    }
    return s;
}

// "key: rest" -> true (key unquoted); the separator is the first ": " or a
// trailing ':' outside quotes.
bool split_key(const std::string& t, std::string* key, std::string* rest) {
    char q = 0;
    for (size_t i = 0; i < t.size(); ++i) {
        const char c = t[i];
        if (q) {
            if (q == '"' && c == '\\') ++i;   // escaped character inside "..."
            else if (c == q) q = 0;
            continue;
        }
        if ((c == '\'' || c == '"') && i == 0) q = c;
        else if (c == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) {
            *key = unquote(rtrim(t.substr(0, i)));
            *rest = i + 1 < t.size() ? t.substr(i + 2) : std::string();
            while (!rest->empty() && rest->front() == ' ') rest->erase(0, 1);
            return true;
        }
    }
    return false;
}

class Parser {
public:
    explicit Parser(const std::string& text) {
        std::istringstream in(text);
        std::string raw;
        while (std::getline(in, raw)) {
            if (raw == "---" || raw == "...") continue;
            std::string s = rtrim(strip_comment(raw));
            size_t ind = 0;
            while (ind < s.size() && s[ind] == ' ') ++ind;
            if (ind == s.size()) continue;
            lines_.push_back({int(ind), s.substr(ind)});
        }
    }
    Node document() {
        if (lines_.empty()) throw ParseError{"empty record"};
        Node n = block(lines_[0].indent);
        if (pos_ != lines_.size()) throw ParseError{"unexpected content at line " + std::to_string(pos_ + 1)};
        return n;
    }

private:
    static bool is_item(const std::string& t) { return t == "-" || t.rfind("- ", 0) == 0; }

    // The record is 5 levels deep; anything far deeper is not a record (and
    // must not exhaust the stack of the recursive descent).
    static constexpr int kMaxDepth = 32;
    int depth_ = 0;

    Node block(int indent) {
        if (pos_ >= lines_.size()) throw ParseError{"missing value"};
        if (++depth_ > kMaxDepth) throw ParseError{"nesting deeper than " + std::to_string(kMaxDepth)};
        Node n = is_item(lines_[pos_].text) ? seq(indent) : map(indent);
        --depth_;
        return n;
    }

    Node seq(int indent) {
        Node n;
        n.kind = Node::Seq;
        while (pos_ < lines_.size() && lines_[pos_].indent == indent && is_item(lines_[pos_].text)) {
            Line& l = lines_[pos_];
            const std::string rest = l.text.size() > 2 ? l.text.substr(2) : std::string();
            if (rest.empty()) {   // "-" alone: the item is the nested block
                ++pos_;
                if (pos_ >= lines_.size() || lines_[pos_].indent <= indent) throw ParseError{"empty sequence item"};
                n.items.push_back(block(lines_[pos_].indent));
                continue;
            }
            std::string k, v;
            if (!(rest.front() == '[' || rest.front() == '!' || rest.front() == '\'' || rest.front() == '"') &&
                split_key(rest, &k, &v)) {
                // "- key: value": a mapping whose first entry shares the dash's line
                l.indent = indent + 2;
                l.text = rest;
                n.items.push_back(map(indent + 2));
                continue;
            }
            ++pos_;
            n.items.push_back(inline_value(rest, indent));
        }
        return n;
    }

    Node map(int indent) {
        Node n;
        n.kind = Node::Map;
        while (pos_ < lines_.size() && lines_[pos_].indent == indent && !is_item(lines_[pos_].text)) {
            std::string k, v;
            if (!split_key(lines_[pos_].text, &k, &v)) throw ParseError{"expected 'key: value': " + lines_[pos_].text};
            ++pos_;
            n.entries.emplace_back(k, inline_value(v, indent));
        }
        return n;
    }

    // The value after "key:" / "- " on the same line; an empty value (or a
    // lone tag) takes the nested block that follows: deeper lines, or an
    // indentless sequence at the parent's indentation.
    Node inline_value(std::string v, int indent) {
        std::string tag;
        if (!v.empty() && v.front() == '!') {
            const size_t sp = v.find(' ');
            tag = v.substr(0, sp);
            v = sp == std::string::npos ? std::string() : v.substr(sp + 1);
            while (!v.empty() && v.front() == ' ') v.erase(0, 1);
        }
        Node n;
        if (v.empty()) {
            if (pos_ < lines_.size() && (lines_[pos_].indent > indent ||
                                         (lines_[pos_].indent == indent && is_item(lines_[pos_].text)))) {
                n = block(lines_[pos_].indent);
            } else {
                n.kind = Node::Scalar;   // null
            }
        } else if (v.front() == '[') {
            n = flow_seq(v);
        } else {
            n.kind = Node::Scalar;
            n.value = unquote(v);
        }
        n.tag = tag;
        return n;
    }

    static Node flow_seq(const std::string& v) {
        if (v.back() != ']') throw ParseError{"unterminated flow sequence: " + v};
        Node n;
        n.kind = Node::Seq;
        std::string body = v.substr(1, v.size() - 2), cur;
        auto push = [&] {
            std::string t = rtrim(cur);
            while (!t.empty() && t.front() == ' ') t.erase(0, 1);
            if (!t.empty()) {
                Node s;
                s.value = unquote(t);
                n.items.push_back(s);
            }
            cur.clear();
        };
        char q = 0;
        for (size_t i = 0; i < body.size(); ++i) {
            const char c = body[i];
            if (q) {
                cur += c;
                if (q == '"' && c == '\\' && i + 1 < body.size()) cur += body[++i];   // escaped character
                else if (c == q) q = 0;
            } else if (c == '\'' || c == '"') {
                q = c;
                cur += c;
            } else if (c == ',') {
                push();
            } else {
                cur += c;
            }
        }
        push();
        return n;
    }

    std::vector<Line> lines_;
    size_t pos_ = 0;
};

uint64_t as_u64(const Node* n, const char* what) {
    if (!n || n->kind != Node::Scalar || n->value.empty()) throw ParseError{std::string("missing field ") + what};
    char* end = nullptr;
    errno = 0;
    const unsigned long long v = std::strtoull(n->value.c_str(), &end, 10);
    if (errno || *end || n->value.front() == '-') throw ParseError{std::string("bad integer in ") + what};
    return v;
}

uint8_t as_u8(const Node& n, const char* what) {
    const uint64_t v = as_u64(&n, what);
    if (v > 255) throw ParseError{std::string(what) + " out of u8 range"};
    return uint8_t(v);
}

std::string as_str(const Node* n, const char* what) {
    if (!n || n->kind != Node::Scalar) throw ParseError{std::string("missing field ") + what};
    return n->value;
}

BlockTopology topology_of(const Node* n) {
    if (!n) throw ParseError{"missing field topology"};
    if (n->kind == Node::Scalar && n->tag.empty() && n->value == "Single") return BlockTopology::single();
    if (n->tag == "!Mirror" && n->kind == Node::Scalar) return BlockTopology::mirror(as_u8(*n, "Mirror"));
    if (n->tag == "!Erasure" && n->kind == Node::Seq && n->items.size() == 3)
        return BlockTopology::erasure(as_u8(n->items[0], "Erasure version"), as_u8(n->items[1], "Erasure data"),
                                      as_u8(n->items[2], "Erasure parity"));
    throw ParseError{"unknown topology variant"};
}

}  // namespace

std::string VirtualFile::to_yaml() const {
    std::ostringstream o;
    o << "ino: " << ino << "\n";
    o << "size: " << size << "\n";
    o << "chunk_size: " << chunk_size << "\n";
    if (blocks.empty()) {
        o << "blocks: []\n";
    } else {
        o << "blocks:\n";
        for (const auto& b : blocks) emit_block(o, b);
    }
    o << "block_size: " << block_size << "\n";
    return o.str();
}

Status VirtualFile::from_yaml(const std::string& text, VirtualFile* out, std::string* err) {
    try {
        Parser p(text);
        const Node doc = p.document();
        if (doc.kind != Node::Map) throw ParseError{"record is not a mapping"};
        VirtualFile vf;
        vf.ino = as_u64(doc.get("ino"), "ino");
        vf.size = as_u64(doc.get("size"), "size");
        vf.chunk_size = as_u64(doc.get("chunk_size"), "chunk_size");
        vf.block_size = as_u64(doc.get("block_size"), "block_size");
        if (vf.chunk_size == 0) throw ParseError{"chunk_size 0"};
        const Node* bl = doc.get("blocks");
        if (!bl || bl->kind != Node::Seq) throw ParseError{"missing field blocks"};
        for (const Node& bn : bl->items) {
            if (bn.kind != Node::Map) throw ParseError{"block is not a mapping"};
            VirtualBlock b;
            b.ino = as_u64(bn.get("ino"), "block ino");
            b.idx = as_u64(bn.get("idx"), "block idx");
            b.size = as_u64(bn.get("size"), "block size");
            b.topology = topology_of(bn.get("topology"));
            const Node* sh = bn.get("shards");
            if (!sh || sh->kind != Node::Seq) throw ParseError{"missing field shards"};
            for (const Node& sn : sh->items) {
                if (sn.kind != Node::Map) throw ParseError{"shard is not a mapping"};
                // named locals, not one braced list: GCC 11 leaks the members a
                // braced aggregate initialiser already built when a later one
                // throws (found by LeakSanitizer on the record fuzz)
                std::string pool = as_str(sn.get("pool"), "pool");
                std::string bucket = as_str(sn.get("bucket"), "bucket");
                std::string filename = as_str(sn.get("filename"), "filename");
                b.shards.push_back({std::move(pool), std::move(bucket), std::move(filename)});
            }
            size_t need = 1;
            if (b.topology.kind == BlockTopology::Mirror) need = b.topology.n;
            if (b.topology.kind == BlockTopology::Erasure) need = size_t(b.topology.data) + b.topology.parity;
            if (b.shards.size() != need) throw ParseError{"block " + std::to_string(b.idx) + ": " +
                                                          std::to_string(b.shards.size()) + " shards for " +
                                                          b.topology.to_string()};
            vf.blocks.push_back(b);
        }
        *out = std::move(vf);
        return std::nullopt;
    } catch (const ParseError& e) {
        if (err) *err = e.what;
        return ShmrError{ShmrError::FsError, EINVAL};
    }
}

Status VirtualFile::save_record(const fs::path& path) const {
    const std::string text = to_yaml();
    const fs::path tmp = path.string() + ".tmp";
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return ShmrError{ShmrError::FsError, errno};
    size_t off = 0;
    while (off < text.size()) {
        const ssize_t n = ::write(fd, text.data() + off, text.size() - off);
        if (n < 0) {
            if (errno == EINTR) continue;
            const int e = errno;
            ::close(fd);
            return ShmrError{ShmrError::FsError, e};
        }
        off += size_t(n);
    }
    if (::fsync(fd) != 0) {
        const int e = errno;
        ::close(fd);
        return ShmrError{ShmrError::FsError, e};
    }
    ::close(fd);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) return ShmrError{ShmrError::FsError, errno};
    return std::nullopt;
}

Status VirtualFile::load_record(const fs::path& path, VirtualFile* out, std::string* err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return ShmrError{ShmrError::FsError, ENOENT};
    std::ostringstream ss;
    ss << f.rdbuf();
    return from_yaml(ss.str(), out, err);
}

}  // namespace shmr
