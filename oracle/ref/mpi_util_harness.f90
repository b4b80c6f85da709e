! mpi_util_harness.f90 — drives the reference's own module_mpi_util under mpirun to produce
! golden vectors for the member <-> column transposes.
!
! TEST INFRASTRUCTURE ONLY (built by oracle/ref/build_mpi_util.sh into oracle/_ref/, run by
! oracle/gen_mpi_util_goldens.py).  Real reference code exercised, compiled unmodified from
! /root/reference: module_mpi_util.f90 (letkf_init, letkf_local_info, letkf_scatter_grid,
! letkf_gather_grid, letkf_scatter_hcoord, letkf_scatter_vcoord, letkf_finalize; MPICH and
! MKL's sgemv underneath), module_config.f90 (read_namelist sets nmember), module_param.f90.
!
! Usage: mpirun -n <nproc> mpi_util_harness <outdir> <nx> <ny> <nz> <k>
! Member m (< k) lives on rank m, as cwb_letkf.f90 reads member files (nproc >= nmember).
! Every rank writes <outdir>/r<rank>.bin (unformatted stream, little-endian):
!   int32  rank, loc_nx, loc_ny, loc_nx_u, loc_ny_v, then xloc, yloc, xloc_u, yloc_v
!   per stagger 0,1,2:   real32 global(gx,gy,nz) input (this rank's member, or rank-id
!                        filler on ranks >= k), local(lx,ly,nz,0:k-1) after scatter_grid,
!                        global(gx,gy,nz) after gather_grid of 2*local (ranks < k)
!   vcoord stagger 0:    ph(nx,ny,nz+1) input, local(loc_nx,loc_ny,nz) after scatter_vcoord
!   vcoord stagger 1:    ph(nx,ny,nz) input, local(loc_nx,loc_ny,nz)
!   vcoord stagger -1:   hgt(nx,ny,1) input (root's is used), local(loc_nx,loc_ny,1)
!   hcoord stagger 0,1,2: lat/lon(gx,gy) input (root's is used), local lat, local lon
! Inputs are integer-valued or dyadic fp32 per (rank, stagger, index), so they are exact.
program mpi_util_harness
    use config,   only : nmember, read_namelist
    use mpi_util
    implicit none
    character(len=512) :: outdir, arg, fname
    integer            :: nx, ny, nz, k, st, gx, gy, lx, ly, nzp
    real, allocatable  :: g3(:,:,:), loc4(:,:,:,:), back(:,:,:), loc3(:,:,:)
    real, allocatable  :: lat(:,:), lon(:,:), llat(:,:), llon(:,:)

    call get_command_argument(1, outdir)
    call get_command_argument(2, arg); read(arg, *) nx
    call get_command_argument(3, arg); read(arg, *) ny
    call get_command_argument(4, arg); read(arg, *) nz
    call get_command_argument(5, arg); read(arg, *) k

    call letkf_init
    ! read_namelist (module_config.f90:79-148) with nmember = k, one file per rank
    write(fname, '(a,"/nml_",i0)') trim(outdir), myid
    open(31, file=trim(fname), status='replace', action='write')
    write(31, '(a)') '&control'
    write(31, '(a,i0)') ' nmember = ', k
    write(31, '(a)') '/'
    write(31, '(a)') '&projection'
    write(31, '(a)') '/'
    write(31, '(a)') '&observations'
    write(31, '(a)') '/'
    write(31, '(a)') '&inflation'
    write(31, '(a)') '/'
    close(31)
    call read_namelist(trim(fname))
    open(31, file=trim(fname), status='old')
    close(31, status='delete')
    if (nmember /= k) stop "mpi_util_harness: nmember not set"

    call letkf_local_info(nx, ny)

    write(fname, '(a,"/r",i0,".bin")') trim(outdir), myid
    open(21, file=trim(fname), access='stream', form='unformatted', status='replace')
    write(21) myid, cpu(myid)%loc_nx, cpu(myid)%loc_ny, cpu(myid)%loc_nx_u, cpu(myid)%loc_ny_v
    write(21) cpu(myid)%xloc, cpu(myid)%yloc, cpu(myid)%xloc_u, cpu(myid)%yloc_v

    ! ---- letkf_scatter_grid / letkf_gather_grid (module_mpi_util.f90:190-358) ----------------
    do st = 0, 2
        gx = nx
        gy = ny
        lx = cpu(myid)%loc_nx
        ly = cpu(myid)%loc_ny
        if (st == 1) then
            gx = nx + 1
            lx = cpu(myid)%loc_nx_u
        end if
        if (st == 2) then
            gy = ny + 1
            ly = cpu(myid)%loc_ny_v
        end if
        allocate(g3(gx, gy, nz), loc4(lx, ly, nz, 0:k-1), back(gx, gy, nz))
        call fill3(g3, 1000 * st + myid)
        loc4 = -7.0
        call letkf_scatter_grid(g3, loc4, st)
        back = -9.0
        call letkf_gather_grid(2.0 * loc4, back, st)
        write(21) g3, loc4, back
        deallocate(g3, loc4, back)
    end do

    ! ---- letkf_scatter_vcoord (:445-580): stagger 0 (destagger), 1 (W/PH levels), -1 (HGT) --
    allocate(loc3(cpu(myid)%loc_nx, cpu(myid)%loc_ny, nz))
    do st = 0, 1
        nzp = nz + 1
        if (st == 1) nzp = nz
        allocate(g3(nx, ny, nzp))
        call fill_ph(g3, 5000 + 10 * st + myid)
        loc3 = -7.0
        call letkf_scatter_vcoord(g3, loc3, st)
        write(21) g3, loc3
        deallocate(g3)
    end do
    deallocate(loc3)
    allocate(g3(nx, ny, 1), loc3(cpu(myid)%loc_nx, cpu(myid)%loc_ny, 1))
    call fill3(g3, 7000 + myid)
    loc3 = -7.0
    call letkf_scatter_vcoord(g3, loc3, -1)
    write(21) g3, loc3
    deallocate(g3, loc3)

    ! ---- letkf_scatter_hcoord (:360-443) ----------------------------------------------------
    do st = 0, 2
        gx = nx
        gy = ny
        lx = cpu(myid)%loc_nx
        ly = cpu(myid)%loc_ny
        if (st == 1) then
            gx = nx + 1
            lx = cpu(myid)%loc_nx_u
        end if
        if (st == 2) then
            gy = ny + 1
            ly = cpu(myid)%loc_ny_v
        end if
        allocate(lat(gx, gy), lon(gx, gy), llat(lx, ly), llon(lx, ly))
        call fill2(lat, 8000 + 10 * st + myid)
        call fill2(lon, 9000 + 10 * st + myid)
        llat = -7.0
        llon = -7.0
        call letkf_scatter_hcoord(lat, llat, lon, llon, st)
        write(21) lat, lon, llat, llon
        deallocate(lat, lon, llat, llon)
    end do
    close(21)

    call letkf_finalize

contains

    ! integer-valued fields: tag * 2^16 + running index (exact in fp32 below 2^24)
    subroutine fill3(a, tag)
        real, intent(out)   :: a(:,:,:)
        integer, intent(in) :: tag
        integer :: i, j, l, n
        n = 0
        do l = 1, size(a, 3)
        do j = 1, size(a, 2)
        do i = 1, size(a, 1)
            a(i, j, l) = real(mod(tag, 200) * 65536 + n)
            n = n + 1
        end do
        end do
        end do
    end subroutine fill3

    subroutine fill2(a, tag)
        real, intent(out)   :: a(:,:)
        integer, intent(in) :: tag
        integer :: i, j, n
        n = 0
        do j = 1, size(a, 2)
        do i = 1, size(a, 1)
            a(i, j) = real(mod(tag, 200)) + real(n) / 1024.0
            n = n + 1
        end do
        end do
    end subroutine fill2

    ! geopotential-like: level * 2937.5 m^2/s^2 plus a dyadic per-rank, per-column spread,
    ! so the ensemble mean's fp32 sums round (sgemv's order matters)
    subroutine fill_ph(a, tag)
        real, intent(out)   :: a(:,:,:)
        integer, intent(in) :: tag
        integer :: i, j, l
        do l = 1, size(a, 3)
        do j = 1, size(a, 2)
        do i = 1, size(a, 1)
            a(i, j, l) = real(l - 1) * 2937.5 + real(mod(tag * 37 + i * 11 + j * 7 + l * 3, 97)) &
                         * 0.7109375 + real(mod(tag, 13)) * 0.0078125
        end do
        end do
        end do
    end subroutine fill_ph

end program mpi_util_harness
