"""Framework-wide constants.

Mirrors the names of the reference (`python/fedml/constants.py:1-34`) so user
configs and code keep working, and adds the MI355X-native simulation type
``RCCL`` (the reference's ``NCCL`` simulator is a stub,
`python/fedml/simulation/simulator.py:100-108`; here ``NCCL`` is accepted as an
alias of ``RCCL`` — on ROCm the torch ``nccl`` backend *is* RCCL).
"""

# training platforms
FEDML_TRAINING_PLATFORM_SIMULATION = "simulation"
FEDML_TRAINING_PLATFORM_CROSS_SILO = "cross_silo"
FEDML_TRAINING_PLATFORM_CROSS_DEVICE = "cross_device"
FEDML_TRAINING_PLATFORM_DISTRIBUTED = "distributed"

# cross-silo scenarios
FEDML_CROSS_SILO_SCENARIO_HORIZONTAL = "horizontal"
FEDML_CROSS_SILO_SCENARIO_HIERARCHICAL = "hierarchical"

# simulation types
FEDML_SIMULATION_TYPE_SP = "single_process"
FEDML_SIMULATION_TYPE_MPI = "MPI"
FEDML_SIMULATION_TYPE_NCCL = "NCCL"
FEDML_SIMULATION_TYPE_RCCL = "RCCL"

# data
FEDML_DATA_CACHE_FOLDER = "fedml_data"
FEDML_DATA_MNIST_URL = "https://fedcv.s3.us-west-1.amazonaws.com/MNIST.zip"

# algorithms
FedML_FEDERATED_OPTIMIZER_BASE_FRAMEWORK = "base_framework"
FedML_FEDERATED_OPTIMIZER_FEDAVG = "FedAvg"
FedML_FEDERATED_OPTIMIZER_S_FEDAVG = "S-FedAvg"
FedML_FEDERATED_OPTIMIZER_HS_FEDAVG = "HS-FedAvg"
FedML_FEDERATED_OPTIMIZER_FEDOPT = "FedOpt"
FedML_FEDERATED_OPTIMIZER_FEDPROX = "FedProx"
FedML_FEDERATED_OPTIMIZER_FEDNOVA = "FedNova"
FedML_FEDERATED_OPTIMIZER_CLASSICAL_VFL = "classical_vertical"
FedML_FEDERATED_OPTIMIZER_SPLIT_NN = "split_nn"
FedML_FEDERATED_OPTIMIZER_DECENTRALIZED_FL = "decentralized_fl"
FedML_FEDERATED_OPTIMIZER_FEDGAN = "FedGAN"
FedML_FEDERATED_OPTIMIZER_FEDAVG_ROBUST = "FedAvg_robust"
FedML_FEDERATED_OPTIMIZER_FEDGKT = "FedGKT"
FedML_FEDERATED_OPTIMIZER_FEDNAS = "FedNAS"
FedML_FEDERATED_OPTIMIZER_FEDSEG = "FedSeg"
FedML_FEDERATED_OPTIMIZER_TURBO_AGGREGATE = "turbo_aggregate"
FedML_FEDERATED_OPTIMIZER_HIERARCHICAL_FL = "HierarchicalFL"

# communication backends (cross-silo / message-passing runtimes)
COMM_BACKEND_LOOPBACK = "LOOPBACK"   # in-process threads (tests, SP-MPI emulation)
COMM_BACKEND_TCP = "TCP"             # native framed sockets (replaces MPI p2p)
COMM_BACKEND_MPI = "MPI"             # accepted: mapped to TCP/loopback (mpi4py not required)
COMM_BACKEND_GRPC = "GRPC"
COMM_BACKEND_TRPC = "TRPC"           # accepted: mapped onto torch.distributed p2p
COMM_BACKEND_MQTT = "MQTT"
COMM_BACKEND_MQTT_S3 = "MQTT_S3"
COMM_BACKEND_MQTT_S3_MNN = "MQTT_S3_MNN"
