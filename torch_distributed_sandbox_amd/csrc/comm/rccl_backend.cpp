// Registration of the native RCCL communicator (implementation: rccl_comm.h).
#include <torch/library.h>

#include "comm/rccl_comm.h"

TORCH_LIBRARY_FRAGMENT(tdsa, m) {
  m.class_<tds_comm::CommWork>("CommWork")
      .def("wait", &tds_comm::CommWork::wait)
      .def("synchronize", &tds_comm::CommWork::synchronize)
      .def("is_completed", &tds_comm::CommWork::is_completed);
  m.class_<tds_comm::RcclComm>("RcclComm")
      .def(torch::init<int64_t, int64_t, int64_t, at::Tensor, int64_t>())
      .def_static("unique_id", &tds_comm::RcclComm::unique_id)
      .def("rank", &tds_comm::RcclComm::rank)
      .def("world_size", &tds_comm::RcclComm::world_size)
      .def("device", &tds_comm::RcclComm::device)
      .def("pending", &tds_comm::RcclComm::pending)
      .def("comm_count", &tds_comm::RcclComm::comm_count)
      .def("cta_budget_min", &tds_comm::RcclComm::cta_budget_min)
      .def("cta_budget_max", &tds_comm::RcclComm::cta_budget_max)
      .def("sendrecv", &tds_comm::RcclComm::sendrecv)
      .def("allreduce", &tds_comm::RcclComm::allreduce)
      .def("broadcast", &tds_comm::RcclComm::broadcast)
      .def("broadcast_coalesced", &tds_comm::RcclComm::broadcast_coalesced)
      .def("reduce", &tds_comm::RcclComm::reduce)
      .def("allgather", &tds_comm::RcclComm::allgather)
      .def("reduce_scatter", &tds_comm::RcclComm::reduce_scatter)
      .def("alltoall", &tds_comm::RcclComm::alltoall)
      .def("send", &tds_comm::RcclComm::send)
      .def("recv", &tds_comm::RcclComm::recv)
      .def("barrier", &tds_comm::RcclComm::barrier)
      .def("abort", &tds_comm::RcclComm::abort)
      .def("shutdown", &tds_comm::RcclComm::shutdown);
}
