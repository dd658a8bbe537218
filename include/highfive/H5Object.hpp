// H5Object.hpp -- HighFive::ObjectType of the read-only HighFive subset over libnr (bits/nr_highfive.hpp).
#pragma once
#include "bits/nr_highfive.hpp"
