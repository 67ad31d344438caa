// gs_host.h — host-side helpers shared by the product library's TUs.
#pragma once
#include <string>

void gs_set_error(const std::string& msg);
