// H5Exception.hpp -- HighFive's exception classes of the read-only HighFive subset over libnr (bits/nr_highfive.hpp).
#pragma once
#include "bits/nr_highfive.hpp"
