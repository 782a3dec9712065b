// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
#include <boost/thread/barrier.hpp>
