// nr_highfive.hpp -- the read-only subset of HighFive (>= 2.1) that the reference's weight
// loaders call, over libnr's HDF5 reader (neural_render.h nr_h5_*).
//
// The reference loads Keras .h5 files through HighFive in NeuralNetwork::load
// (src/neuralNetwork.cpp:86-129) and simpleInfer's loadModelFromH5 (src/simpleInfer.cpp:13-79):
//   File(fp, File::ReadOnly), listObjectNames(), getObjectType(name), getGroup(name),
//   Group::getNumberObjects(), getDataSet(name), DataSet::getDimensions(),
//   DataSet::read(std::vector<float>&) and read(std::vector<std::vector<float>>&).
// Those calls compile unchanged against this header (include path only; link libnr).
// Everything else HighFive offers (writing, attributes, properties, other types) is not
// here.  Errors throw HighFive's exception classes with the reader's message.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../neural_render.h"

namespace HighFive {

enum class ObjectType { File, Group, UserDataType, DataSpace, Dataset, Attribute, Other };

class Exception : public std::exception {
  public:
    explicit Exception(const std::string &msg) : msg_(msg) {}
    const char *what() const noexcept override { return msg_.c_str(); }
    const std::string &getErrMsg() const { return msg_; }

  private:
    std::string msg_;
};
class FileException : public Exception { using Exception::Exception; };
class ObjectException : public Exception { using Exception::Exception; };
class GroupException : public Exception { using Exception::Exception; };
class DataSetException : public Exception { using Exception::Exception; };
class DataSpaceException : public Exception { using Exception::Exception; };

class Group;
class DataSet;

namespace detail {

using Handle = std::shared_ptr<nr_h5_file>;

template <class E>
inline void check(int rc, const std::string &what) {
    if (rc != NR_OK) throw E(what + ": " + nr_last_error(nullptr));
}

// Group-like objects (File, Group): HighFive's NodeTraits
template <class Derived>
class NodeTraits {
  public:
    size_t getNumberObjects() const {
        size_t n = 0;
        check<GroupException>(nr_h5_num_members(h_.get(), id_, &n), "Unable to count objects in group");
        return n;
    }
    std::string getObjectName(size_t index) const {
        size_t len = 0;
        check<GroupException>(nr_h5_member(h_.get(), id_, index, nullptr, 0, &len, nullptr), "Unable to get object name");
        std::string s(len + 1, '\0');
        check<GroupException>(nr_h5_member(h_.get(), id_, index, &s[0], s.size(), nullptr, nullptr),
                              "Unable to get object name");
        s.resize(len);
        return s;
    }
    // member names in HDF5 name order ("dense_10" before "dense_2"), as HighFive returns them
    std::vector<std::string> listObjectNames() const {
        std::vector<std::string> names;
        const size_t n = getNumberObjects();
        names.reserve(n);
        for (size_t i = 0; i < n; ++i) names.push_back(getObjectName(i));
        return names;
    }
    bool exist(const std::string &name) const {
        uint64_t obj = 0;
        return find(name, obj);
    }
    ObjectType getObjectType(const std::string &name) const {
        const uint64_t obj = member(name, "Unable to get the type of object");
        int t = NR_H5_OTHER;
        check<ObjectException>(nr_h5_object_type(h_.get(), obj, &t), "Unable to get the type of object " + name);
        return t == NR_H5_GROUP ? ObjectType::Group : (t == NR_H5_DATASET ? ObjectType::Dataset : ObjectType::Other);
    }
    inline Group getGroup(const std::string &name) const;
    inline DataSet getDataSet(const std::string &name) const;

  protected:
    NodeTraits(Handle h, uint64_t id) : h_(std::move(h)), id_(id) {}
    bool find(const std::string &name, uint64_t &obj) const {
        const size_t n = getNumberObjects();
        for (size_t i = 0; i < n; ++i)
            if (getObjectName(i) == name) {
                check<GroupException>(nr_h5_member(h_.get(), id_, i, nullptr, 0, nullptr, &obj), "Unable to open object");
                return true;
            }
        return false;
    }
    uint64_t member(const std::string &name, const std::string &what) const {
        uint64_t obj = 0;
        if (!find(name, obj)) throw GroupException(what + " \"" + name + "\": no such object");
        return obj;
    }
    int type_of(uint64_t obj) const {
        int t = NR_H5_OTHER;
        check<ObjectException>(nr_h5_object_type(h_.get(), obj, &t), "Unable to get the type of object");
        return t;
    }

    Handle h_;
    uint64_t id_;
};

}  // namespace detail

class DataSpace {
  public:
    explicit DataSpace(std::vector<size_t> dims) : dims_(std::move(dims)) {}
    size_t getNumberDimensions() const { return dims_.size(); }
    std::vector<size_t> getDimensions() const { return dims_; }
    size_t getElementCount() const {
        size_t n = 1;
        for (size_t d : dims_) n *= d;
        return n;
    }

  private:
    std::vector<size_t> dims_;
};

class DataSet {
  public:
    std::vector<size_t> getDimensions() const {
        int nd = 0;
        detail::check<DataSetException>(nr_h5_dims(h_.get(), id_, nullptr, 0, &nd), "Unable to get dataspace");
        std::vector<uint64_t> d((size_t)nd);
        detail::check<DataSetException>(nr_h5_dims(h_.get(), id_, d.data(), nd, &nd), "Unable to get dataspace");
        return std::vector<size_t>(d.begin(), d.end());
    }
    DataSpace getSpace() const { return DataSpace(getDimensions()); }
    size_t getElementCount() const { return getSpace().getElementCount(); }

    // 1-D (or N-D with at most one dimension != 1) into a flat vector
    void read(std::vector<float> &out) const {
        const auto dims = getDimensions();
        size_t big = 0;
        for (size_t d : dims) big += d != 1;
        if (big > 1)
            throw DataSpaceException("Impossible to read DataSet of dimensions " + std::to_string(dims.size()) +
                                     " into arrays of dimensions 1");
        out.resize(getElementCount());
        detail::check<DataSetException>(nr_h5_read_f32(h_.get(), id_, out.data(), out.size()), "Unable to read dataset");
    }
    // 2-D into rows (Keras kernels: rows = inputs, columns = outputs)
    void read(std::vector<std::vector<float>> &out) const {
        const auto dims = getDimensions();
        if (dims.size() != 2)
            throw DataSpaceException("Impossible to read DataSet of dimensions " + std::to_string(dims.size()) +
                                     " into arrays of dimensions 2");
        std::vector<float> flat(dims[0] * dims[1]);
        detail::check<DataSetException>(nr_h5_read_f32(h_.get(), id_, flat.data(), flat.size()), "Unable to read dataset");
        out.assign(dims[0], std::vector<float>(dims[1]));
        for (size_t r = 0; r < dims[0]; ++r)
            for (size_t c = 0; c < dims[1]; ++c) out[r][c] = flat[r * dims[1] + c];
    }

  private:
    template <class> friend class detail::NodeTraits;
    DataSet(detail::Handle h, uint64_t id) : h_(std::move(h)), id_(id) {}
    detail::Handle h_;
    uint64_t id_;
};

class Group : public detail::NodeTraits<Group> {
  private:
    template <class> friend class detail::NodeTraits;
    Group(detail::Handle h, uint64_t id) : NodeTraits(std::move(h), id) {}
};

class File : public detail::NodeTraits<File> {
  public:
    enum : unsigned {
        ReadOnly = 0x00u,
        ReadWrite = 0x01u,
        Truncate = 0x02u,
        Excl = 0x04u,
        Debug = 0x08u,
        Create = 0x10u,
        Overwrite = Truncate,
        OpenOrCreate = ReadWrite | Create
    };
    explicit File(const std::string &filename, unsigned openFlags = ReadOnly)
        : NodeTraits(open(filename, openFlags), 0), name_(filename) {
        detail::check<FileException>(nr_h5_root(h_.get(), &id_), "Unable to open file " + filename);
    }
    const std::string &getName() const { return name_; }

  private:
    static detail::Handle open(const std::string &filename, unsigned flags) {
        if (flags != ReadOnly) throw FileException("Unable to open file " + filename + ": this HighFive subset is read-only");
        nr_h5_file *f = nullptr;
        detail::check<FileException>(nr_h5_open(filename.c_str(), &f), "Unable to open file " + filename);
        return detail::Handle(f, nr_h5_close);
    }
    std::string name_;
};

template <class Derived>
inline Group detail::NodeTraits<Derived>::getGroup(const std::string &name) const {
    const uint64_t obj = member(name, "Unable to open the group");
    if (type_of(obj) != NR_H5_GROUP) throw GroupException("Unable to open the group \"" + name + "\": not a group");
    return Group(h_, obj);
}

template <class Derived>
inline DataSet detail::NodeTraits<Derived>::getDataSet(const std::string &name) const {
    const uint64_t obj = member(name, "Unable to open the dataset");
    if (type_of(obj) != NR_H5_DATASET) throw DataSetException("Unable to open the dataset \"" + name + "\": not a dataset");
    return DataSet(h_, obj);
}

}  // namespace HighFive
