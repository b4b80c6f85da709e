! ingest_driver.f90 — a Fortran host reading one cycle's member obs files through the core's
! ingest (include/cwb_letkf_ingest.h), as cwb_letkf.f90:46-57 would after the edit in
! INTEGRATION.md §1.0: every member's gts_letkf_### / VR_letkf_### / MR_letkf_### file, then
! the one-buffer wire image of the set, written raw to the output file.  Used by
! tests/test_fortran_host.py (no GPU needed: the ingest is host code).
!
! usage: ingest_driver <dir> <nmember> <out.bin>
program ingest_driver
    use iso_c_binding
    use letkf_core_gpu
    implicit none
    character(len=512) :: dir, arg, out
    character(len=3)   :: mm
    integer            :: k, m, u
    type(c_ptr)        :: h
    type(cwbl_projection) :: proj
    type(cwbl_obs_set)    :: os
    integer(c_long_long)  :: nw
    real(c_float), allocatable :: wire(:)

    call get_command_argument(1, dir)
    call get_command_argument(2, arg)
    call get_command_argument(3, out)
    read (arg, *) k
    proj = cwbl_projection(120.0, 23.7644, 10.0, 40.0)   ! projection_nml defaults
    h = cwbl_ingest_create(int(k, c_int), proj)
    if (.not. c_associated(h)) call cwbl_check(1_c_int, 'cwbl_ingest_create')
    do m = 1, k
        write (mm, '(i3.3)') m
        call cwbl_check(cwbl_ingest_read_gts(h, -1_c_int, trim(dir)//'/gts_letkf_'//mm//c_null_char, &
                                             trim(dir)//'/obs_gts'//c_null_char), 'read_gts')
        call cwbl_check(cwbl_ingest_read_radar(h, -1_c_int, trim(dir)//'/VR_letkf_'//mm//c_null_char, &
                                               'VR'//c_null_char), 'read_radar VR')
        call cwbl_check(cwbl_ingest_read_radar(h, -1_c_int, trim(dir)//'/MR_letkf_'//mm//c_null_char, &
                                               'MR'//c_null_char), 'read_radar MR')
    end do
    call cwbl_check(cwbl_ingest_obs_set(h, os), 'obs_set')
    nw = cwbl_ingest_wire_words(h)
    allocate(wire(nw))
    call cwbl_check(cwbl_ingest_pack_wire(h, wire, nw), 'pack_wire')
    open (newunit=u, file=trim(out), access='stream', form='unformatted', status='replace')
    write (u) wire
    close (u)
    print '(a,i0,a,i0,a,i0)', 'fortran ingest: gts types=', os%n_gts, ' radar types=', os%n_radar, &
        ' words=', nw
    call cwbl_ingest_destroy(h)
end program ingest_driver
