// Registration of the native host ring communicator (implementation: host_comm.h).
#include <torch/library.h>

#include "comm/host_comm.h"

TORCH_LIBRARY_FRAGMENT(tdsa, m) {
  m.class_<tds_comm::HostComm>("HostComm")
      .def(torch::init<int64_t, int64_t, int64_t>())
      .def("port", &tds_comm::HostComm::port)
      .def("rank", &tds_comm::HostComm::rank)
      .def("world_size", &tds_comm::HostComm::world_size)
      .def("connect", &tds_comm::HostComm::connect)
      .def("allreduce_", &tds_comm::HostComm::allreduce_)
      .def("reduce_scatter_", &tds_comm::HostComm::reduce_scatter_)
      .def("broadcast_", &tds_comm::HostComm::broadcast_)
      .def("allgather", &tds_comm::HostComm::allgather)
      .def("barrier", &tds_comm::HostComm::barrier)
      .def("close", &tds_comm::HostComm::close_all);
}
