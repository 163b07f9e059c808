// ChannelFsm mirror: the part of src/algorithms/channel/libs/channel_fsm.h:41-81
// that the acquisition block calls.  The reference block holds a
// std::weak_ptr<ChannelFsm> (set through AcquisitionInterface::set_channel_fsm,
// acquisition_interface.h:53, which Channel's constructor calls, channel.cc:50)
// and on a positive acquisition calls Event_valid_acquisition() directly instead
// of publishing event 1 (pcps_acquisition.cc:370-377).  The channel FSM itself
// (states, tracking start, satellite requests) is the caller's and out of scope
// (SURVEY.md §2); a maintainer building the adapters against the reference tree
// includes the reference's channel_fsm.h in place of this header.
#ifndef GSDR_HOST_CHANNEL_FSM_H
#define GSDR_HOST_CHANNEL_FSM_H

class ChannelFsm
{
public:
    virtual ~ChannelFsm() = default;
    // FSM events the acquisition / tracking blocks fire (channel_fsm.h:56-62)
    virtual bool Event_valid_acquisition() { return true; }
    virtual bool Event_failed_acquisition_repeat() { return true; }
    virtual bool Event_failed_acquisition_no_repeat() { return true; }
};

#endif
