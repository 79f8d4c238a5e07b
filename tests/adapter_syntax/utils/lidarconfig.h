// include/utils/lidarconfig.h:7-56 (the fields the adapter reads; defaults as there).
#pragma once
struct lidarConfig {
  bool using_sharp_point = true;
  bool using_flat_point = true;
  double distance_sq_threshold = 0.2;
  double flat_optimized_weight = 50;
};
