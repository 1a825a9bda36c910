// fmi.h — umbrella header (mirrors reference include/fmi.h): the Communicator plus the bundled channels.
#ifndef FMI_AMD_FMI_H
#define FMI_AMD_FMI_H

#include "Communicator.h"
#include "comm/LocalSocket.h"
#include "comm/Loopback.h"
#include "comm/PeerToPeer.h"
#include "comm/Rccl.h"

#endif
