// FMI::Utils::Configuration — reads the reference's JSON configuration schema (config/fmi.json:
// "backends" {name: {enabled, host, port, ...}}, "model" {name: {...}, "FaaS": {gib_second_price}}) and
// returns the enabled backends with their model parameters (reference src/utils/Configuration.cpp:12-42).
// The reference parses with boost::property_tree (absent here); this is a small self-contained reader of
// the JSON subset the schema uses (objects, strings, numbers, booleans; arrays are skipped). Values are
// returned as strings, exactly as property_tree's data() hands them to the channel factories.
#ifndef FMI_AMD_UTILS_CONFIGURATION_H
#define FMI_AMD_UTILS_CONFIGURATION_H

#include <cctype>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>

namespace FMI::Utils {

class Configuration {
public:
    using Params = std::map<std::string, std::string>;
    using Backends = std::map<std::string, std::pair<Params, Params>>;

    explicit Configuration(const std::string& config_path) {
        std::ifstream in(config_path);
        if (!in) throw std::runtime_error(config_path + ": cannot open FMI configuration");
        std::stringstream ss;
        ss << in.rdbuf();
        text_ = ss.str();
        pos_ = 0;
        root_ = parse_value();
    }

    //! Enabled backends: name -> (backend params, model params).
    Backends get_active_channels() const {
        Backends out;
        const Node* backends = root_.child("backends");
        const Node* model = root_.child("model");
        if (!backends) return out;
        for (const auto& [name, node] : backends->members) {
            Params params = node->flatten();
            auto it = params.find("enabled");
            if (it != params.end() && it->second != "true") continue;
            Params model_params;
            if (model && model->child(name)) model_params = model->child(name)->flatten();
            out[name] = {params, model_params};
        }
        return out;
    }

    //! FaaS price per GiB-second (model.FaaS.gib_second_price).
    double get_faas_price() const {
        const Node* model = root_.child("model");
        const Node* faas = model ? model->child("FaaS") : nullptr;
        const Node* price = faas ? faas->child("gib_second_price") : nullptr;
        if (!price) throw std::runtime_error("configuration lacks model.FaaS.gib_second_price");
        return std::stod(price->scalar);
    }

private:
    struct Node {
        std::string scalar;  // leaf value as text
        std::map<std::string, std::shared_ptr<Node>> members;
        bool object = false;
        const Node* child(const std::string& k) const {
            auto it = members.find(k);
            return it == members.end() ? nullptr : it->second.get();
        }
        Params flatten() const {
            Params p;
            for (const auto& [k, v] : members)
                if (!v->object) p[k] = v->scalar;
            return p;
        }
    };

    void ws() {
        while (pos_ < text_.size() && std::isspace(static_cast<unsigned char>(text_[pos_]))) ++pos_;
    }
    [[noreturn]] void bad(const char* what) const {
        throw std::runtime_error(std::string("configuration JSON: ") + what + " at offset " + std::to_string(pos_));
    }
    std::string parse_string() {
        if (text_[pos_] != '"') bad("expected string");
        ++pos_;
        std::string s;
        while (pos_ < text_.size() && text_[pos_] != '"') {
            if (text_[pos_] == '\\' && pos_ + 1 < text_.size()) ++pos_;
            s += text_[pos_++];
        }
        if (pos_ >= text_.size()) bad("unterminated string");
        ++pos_;
        return s;
    }
    Node parse_value() {
        ws();
        if (pos_ >= text_.size()) bad("unexpected end");
        Node n;
        const char c = text_[pos_];
        if (c == '{') {
            n.object = true;
            ++pos_;
            ws();
            if (text_[pos_] == '}') {
                ++pos_;
                return n;
            }
            while (true) {
                ws();
                std::string key = parse_string();
                ws();
                if (text_[pos_] != ':') bad("expected ':'");
                ++pos_;
                n.members[key] = std::make_shared<Node>(parse_value());
                ws();
                if (text_[pos_] == ',') {
                    ++pos_;
                    continue;
                }
                if (text_[pos_] == '}') {
                    ++pos_;
                    return n;
                }
                bad("expected ',' or '}'");
            }
        }
        if (c == '[') {  // not used by the schema: skip balanced
            int depth = 0;
            do {
                if (text_[pos_] == '[') ++depth;
                if (text_[pos_] == ']') --depth;
                ++pos_;
            } while (depth > 0 && pos_ < text_.size());
            return n;
        }
        if (c == '"') {
            n.scalar = parse_string();
            return n;
        }
        const std::size_t start = pos_;
        while (pos_ < text_.size() && (std::isalnum(static_cast<unsigned char>(text_[pos_])) || text_[pos_] == '.' ||
                                       text_[pos_] == '-' || text_[pos_] == '+'))
            ++pos_;
        if (start == pos_) bad("unexpected character");
        n.scalar = text_.substr(start, pos_ - start);
        return n;
    }

    std::string text_;
    std::size_t pos_ = 0;
    Node root_;
};

}  // namespace FMI::Utils

#endif
