// Minimal ConfigurationInterface / InMemoryConfiguration mirror
// (src/core/interfaces/configuration_interface.h:44-59,
//  src/core/receiver/in_memory_configuration.cc): string properties with typed
// property(name, default) lookups, as the adapters use them.
#ifndef GSDR_HOST_CONFIGURATION_H
#define GSDR_HOST_CONFIGURATION_H

#include <cstdint>
#include <map>
#include <sstream>
#include <string>

class ConfigurationInterface
{
public:
    virtual ~ConfigurationInterface() = default;
    virtual std::string property(const std::string& name, const std::string& default_value) const = 0;
    virtual void set_property(const std::string& name, const std::string& value) = 0;

    template <typename T>
    T property(const std::string& name, T default_value) const
    {
        const std::string s = property(name, std::string());
        if (s.empty()) return default_value;
        std::istringstream is(s);
        T v{};
        if (!(is >> v)) return default_value;
        return v;
    }
    bool property(const std::string& name, bool default_value) const
    {
        const std::string s = property(name, std::string());
        if (s.empty()) return default_value;
        return s == "true" || s == "1" || s == "TRUE" || s == "True";
    }
    std::string property(const std::string& name, const char* default_value) const
    {
        return property(name, std::string(default_value));
    }
};

class InMemoryConfiguration : public ConfigurationInterface
{
public:
    std::string property(const std::string& name, const std::string& default_value) const override
    {
        auto it = props_.find(name);
        return it == props_.end() ? default_value : it->second;
    }
    using ConfigurationInterface::property;
    void set_property(const std::string& name, const std::string& value) override { props_[name] = value; }

private:
    std::map<std::string, std::string> props_;
};

#endif
